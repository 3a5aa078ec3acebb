// tuning.h -- the launch-shape constants chosen by measurement, in one place.
//
// Each value below was picked by an A/B on the MI355X (records under profiles/, DESIGN.md section
// 4); the alternatives lost and their code paths were deleted.  These are the only compile-time
// knobs in the product sources: tools/build_variants.py may override one with -D to rebuild a
// variant library for a new A/B, the product build never does.
#pragma once

// gemm_f64_kernel (fp64 panel path): waves per block, 32 samples each (profiles/r4f, r4g)
#ifndef GPDLA_F64_WAVES
#define GPDLA_F64_WAVES 4
#endif

// gemm_i8_bst_kernel: XCDs sharing a sample tile's A digits (4 / 8 measured -1.3% / -5%, profiles/r5j)
#ifndef GPDLA_BST_EX
#define GPDLA_BST_EX 2
#endif

// panel paths: largest sample chunk per spectrum (2 / 4 / 6 equal chunks lost 2-15%, profiles/r2/c5_ab, r7e)
#ifndef GPDLA_MAX_CHUNK
#define GPDLA_MAX_CHUNK 131072
#endif

// gemm_i8_bst_kernel: share of an XCD's u sample tiles taken by its two spare blocks (the Gram
// blocks take the rest after their columns); configs[4]: 0.15 / 0.25 / 0.35 / 0.40 / 0.45 / 0.50 /
// 0.55 / 0.65 -> 9.96 / 9.97 / 9.99 / 10.08 / 10.03 / 9.79 / 9.44 / 8.93e7 evals/s (profiles/round5/r10h-j)
#ifndef GPDLA_BST_USPARE
#define GPDLA_BST_USPARE 0.40f
#endif
