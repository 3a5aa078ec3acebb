/* gpdla.h -- C ABI of the MI355X GP-DLA likelihood engine (libgpdla.so).
 *
 * Drop-in boundary for the hot path of sbird/gp_dla_detection (paths are relative to the
 * reference repository):
 *
 *   reference interface                                  replaced by
 *   ---------------------------------------------------  -------------------------------------
 *   voigt MEX: absorption = voigt(lambdas, z, N, nl)     gpdla_voigt_f64
 *     (voigt.c:253-304, called at process_qsos.m:186)
 *   log_p = log_mvnpdf_low_rank(y, mu, M, d)             gpdla_log_mvnpdf_low_rank_f64
 *     (log_mvnpdf_low_rank.m:5-33, process_qsos.m:151,196)
 *   process_qsos.m:88-220 per-spectrum loop + parfor    gpdla_engine_create / _process /
 *     over DLA samples (process_qsos.m:184-198)            _synchronize / _destroy
 *   generate_dla_samples.m:8-57 (haltonset/scramble,     gpdla_generate_dla_samples_f64,
 *     ksdensity, polyfit, integral, fzero)                 gpdla_halton_rr2_f64
 *   read_spec.m:27-38, preload_qsos.m:18-67              gpdla_read_spec_f32,
 *                                                          gpdla_preload_qsos_f32
 *
 * Conventions
 *   - Plain pointers and sizes only.  The caller owns every buffer; the engine owns only its
 *     device workspaces.  Nothing allocated by the library is returned across the ABI.
 *   - Matrices follow MATLAB: M is (rows x k) COLUMN-major.
 *   - Every function returns an int status: GPDLA_OK (0), a negative error, or GPDLA_ENUMERIC
 *     (a non-positive Cholesky/LDL pivot or a non-finite value was met; the affected outputs
 *     are NaN -- MATLAB's chol would have raised, log_mvnpdf_low_rank.m:24).
 *     A message is available from gpdla_last_error() (thread-local).
 *   - Reentrant.  One engine is driven by one host thread; engines on different devices (or
 *     the same device) may run concurrently.
 *   - There is no CPU fallback: without a usable HIP device every compute entry point fails
 *     with GPDLA_EDEVICE.
 */
#ifndef GPDLA_H
#define GPDLA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPDLA_OK 0
#define GPDLA_ENUMERIC 1
#define GPDLA_EINVAL (-1)
#define GPDLA_EDEVICE (-2)
#define GPDLA_ENOMEM (-3)
#define GPDLA_EUNSUPPORTED (-4)

/* ABI version (gpdla_version()).  2: gpdla_stats gained contraction_ms / contraction_launches
 * (its size changed: a caller compiled against a version-1 header must use gpdla_engine_get_stats_n
 * with its own sizeof(gpdla_stats), or be rebuilt).  3: gpdla_device_pci_bus_id.  4: the DLA-sample
 * generator (gpdla_halton_rr2_f64, gpdla_generate_dla_samples_f64) and the ingest kernels.
 * 5: gpdla_last_call_kernel_ms. */
#define GPDLA_ABI_VERSION 5

#define GPDLA_MEM_HOST 0
#define GPDLA_MEM_DEVICE 1

/* absorption-index handling (process_qsos.m:180,189) */
#define GPDLA_ABSORPTION_REFERENCE 0 /* reproduce the quirk: absorption(1:n) of the m in-range values */
#define GPDLA_ABSORPTION_UNMASKED 1  /* pair every unmasked pixel with its own profile value */
/* Likelihood path.  AUTO = the fused single-kernel sweep for ranks 1..24 (compiled for 4 8 10 12 16
 * 20 24; a rank in between runs on the next compiled one with M padded by zero columns, which is
 * exact: pivots 1, zero updates), otherwise the panel-GEMM path (weights kernel + fp64 Gram/u GEMM +
 * batched LDL^T), which takes any rank 1..64 (BASELINE configs[4]: k = 50). */
#define GPDLA_PATH_AUTO 0
#define GPDLA_PATH_FUSED 1
#define GPDLA_PATH_PANEL_GEMM 2
/* Fused sweep with the Gram/u contraction on the int8 matrix cores (Ozaki digit slicing: 32-bit
 * quantised operands, exact integer accumulation, fp64 everywhere else); k <= 20 (compiled for 20,
 * lower ranks zero-padded) with num_lines = 3.  Spectra with more than 30,000 pixels fall back to the
 * fp64 fused kernel.  Agrees with the fp64 path to <= 4e-9 relative on the log-likelihoods (measured
 * 3.8e-9 at BASELINE configs[1]; tests assert 1e-8). */
#define GPDLA_PATH_FUSED_I8 3
/* Panel-GEMM path with the Gram/u GEMMs on the int8 matrix cores (same Ozaki scheme as
 * GPDLA_PATH_FUSED_I8), any rank 1..64 with num_lines = 3; for BASELINE configs[4] (k = 50, quoted in
 * fp32) it agrees with fp64 to <= 4e-9 relative (tests assert 1e-8), far inside fp32's ~5e-6. */
#define GPDLA_PATH_PANEL_GEMM_I8 4
/* GPDLA_PATH_PANEL_GEMM_I8 with a 24-bit Gram contraction: 3 digit planes per operand and the 6 digit
 * pairs of level <= 2 for the k(k+1)/2 Gram entries (instead of 4 planes and 10 pairs: 40% fewer
 * matrix-core operations); the k u entries keep the 32-bit scheme.  Fp32-class, as BASELINE configs[4]
 * is quoted (an fp32 Gram/Cholesky gives 4.5-6e-6): a few 1e-7 relative from fp64 on
 * the log-likelihoods at k = 50, inside the 1e-6 contract. */
#define GPDLA_PATH_PANEL_GEMM_I8_24 5

/* Learned null model (learned_qso_model_<set>.mat, read at process_qsos.m:30-35).  Host memory. */
typedef struct gpdla_model {
  int32_t num_rest;              /* rest-grid size (1,217 for 911.75:0.25:1215.75) */
  int32_t k;                     /* rank (set_parameters.m:36) */
  const double* rest_wavelengths;/* [num_rest], strictly increasing */
  const double* mu;              /* [num_rest] */
  const double* M;               /* [num_rest x k], column-major */
  const double* log_omega;       /* [num_rest] */
  double log_c_0, log_tau_0, log_beta;
} gpdla_model;

/* DLA parameter samples (dla_samples.mat, read at process_qsos.m:38-40).  Host memory. */
typedef struct gpdla_samples {
  int64_t num_samples;           /* S (set_parameters.m:48) */
  const double* offset_samples;  /* [S] in [0,1] */
  const double* nhi_samples;     /* [S] N_HI in cm^-2 (10.^log_nhi_samples) */
} gpdla_samples;

/* set_parameters.m knobs the path reads. */
typedef struct gpdla_params {
  int32_t num_lines;             /* 1..31 (set_parameters.m:63; voigt.c:16) */
  int32_t width;                 /* must be 3 (set_parameters.m:59 == voigt.c:229) */
  double pixel_spacing;          /* 1e-4 dex (set_parameters.m:60) */
  double min_lambda, max_lambda; /* 911.75, 1215.75 (set_parameters.m:33-34) */
  double lya_wavelength;         /* 1215.6701 (set_parameters.m:5) */
  double lyman_limit;            /* 911.7633 (set_parameters.m:7) */
  double min_z_cut, max_z_cut;   /* kms_to_z(3000) (set_parameters.m:65,69) */
  int32_t absorption_mode;       /* GPDLA_ABSORPTION_* */
  int32_t max_batch_spectra;     /* spectra per device batch; 0 = library default */
  int32_t path;                  /* GPDLA_PATH_*: fused kernel or panel-GEMM (see below) */
} gpdla_params;

/* Preloaded spectra (preloaded_qsos.mat cells, process_qsos.m:46-61), CSR-packed.
 * `offsets` is ALWAYS host memory; the pixel arrays and z_qsos live in `memory`. */
typedef struct gpdla_spectra {
  int32_t memory;                /* GPDLA_MEM_HOST or GPDLA_MEM_DEVICE */
  int64_t num_spectra;           /* Q */
  const int64_t* offsets;        /* [Q+1] host; spectrum q = pixels offsets[q]..offsets[q+1]-1 */
  const double* wavelengths;     /* observed, Angstrom */
  const double* flux;
  const double* noise_variance;
  const uint8_t* pixel_mask;     /* nonzero = masked */
  const double* z_qsos;          /* [Q] */
} gpdla_spectra;

/* Per-spectrum outputs (the hot-path subset of processed_qsos_<set>.mat, process_qsos.m:235-249). */
typedef struct gpdla_results {
  int32_t memory;                      /* GPDLA_MEM_HOST or GPDLA_MEM_DEVICE */
  double* log_likelihoods_no_dla;      /* [Q]   process_qsos.m:150-152 */
  double* sample_log_likelihoods_dla;  /* [Q x sample_ld] spectrum-major, or NULL (process_qsos.m:195) */
  int64_t sample_ld;                   /* >= S */
  double* log_likelihoods_dla;         /* [Q]   process_qsos.m:202-209 */
  double* min_z_dlas;                  /* [Q]   process_qsos.m:160 (may be NULL) */
  double* max_z_dlas;                  /* [Q]   process_qsos.m:161 (may be NULL) */
  int32_t* num_pixels;                 /* [Q]   n, unmasked in-range pixels (may be NULL) */
} gpdla_results;

/* Kernel-time accounting (HIP events on the engine's stream), cumulative since create/reset.
 * likelihood_ms spans each batch's likelihood work on the engine's stream.  contraction_ms is the sum
 * of the event spans around each Gram/u GEMM launch (panel-GEMM paths): with one panel stream those
 * spans lie inside likelihood_ms; with panel_streams > 1 the launches of different streams overlap in
 * time and each span also counts the time its launch waits behind the other streams' kernels, so the
 * sum is not part of likelihood_ms and can exceed it (set 1 panel stream to time the kernel alone). */
typedef struct gpdla_stats {
  double prep_ms, likelihood_ms, reduce_ms;
  int64_t prep_launches, likelihood_launches, reduce_launches;
  int64_t spectra, sample_evals;       /* sample_evals = sum over spectra of S (null evals excluded) */
  double contraction_ms;               /* panel-GEMM paths: summed GEMM launch spans (see above) */
  int64_t contraction_launches;
} gpdla_stats;

typedef struct gpdla_engine gpdla_engine;

int gpdla_engine_create(int32_t device, const gpdla_model* model, const gpdla_samples* samples,
                        const gpdla_params* params, gpdla_engine** out);
/* Enqueue the whole pipeline for all spectra.  With GPDLA_MEM_HOST results the call blocks until
 * the outputs are copied back; with device results it returns after enqueueing (use
 * gpdla_engine_synchronize).  Spectra may be processed in several device batches.  With host
 * inputs and host results the batches are pipelined: batch b's inputs are copied in, and batch
 * b - 1's results copied out, on a copy stream of the engine's own while the kernels run. */
int gpdla_engine_process(gpdla_engine* engine, const gpdla_spectra* spectra,
                         const gpdla_results* results);
/* Wait for enqueued work; returns GPDLA_ENUMERIC if any pivot was non-positive since the last call. */
int gpdla_engine_synchronize(gpdla_engine* engine);
/* Use an external hipStream_t (NULL restores the engine's own stream; the null stream itself is
 * selected by gpdla_engine_use_null_stream).  All kernels of a process
 * call are ordered on that stream (after the work already on it); the host-buffer copies above run on
 * the engine's copy stream, ordered against it by events. */
int gpdla_engine_set_stream(gpdla_engine* engine, void* hip_stream);
/* Order the kernels on the null stream (stream 0, e.g. PyTorch's default stream), as
 * gpdla_engine_set_stream does for any other stream. */
int gpdla_engine_use_null_stream(gpdla_engine* engine);
/* Panel-GEMM paths (fp64 and int8): the number of compute streams (1..4, default 2) a batch's spectra
 * alternate over.  Spectrum q of a batch runs on stream q % n (0 = the engine's stream, the others
 * engine-owned) with a workspace of its own, forked from and joined back into the engine's stream;
 * results are bitwise identical for every n. */
int gpdla_engine_set_panel_streams(gpdla_engine* engine, int32_t n);
int gpdla_engine_get_stats(gpdla_engine* engine, gpdla_stats* stats);
/* The same, writing at most stats_bytes bytes (a caller's sizeof(gpdla_stats) from an older header). */
int gpdla_engine_get_stats_n(gpdla_engine* engine, gpdla_stats* stats, int64_t stats_bytes);
int gpdla_engine_reset_stats(gpdla_engine* engine);
void gpdla_engine_destroy(gpdla_engine* engine);

/* voigt MEX replacement (voigt.c:253-304).  Host buffers.  out has n_padded - 6 values. */
int gpdla_voigt_f64(const double* lambdas, int64_t n_padded, double z, double N,
                    int32_t num_lines, double* out);
/* Batched form: out[s*(n_padded-6) + i] for `count` (z, N) pairs over one padded grid. */
int gpdla_voigt_batch_f64(const double* lambdas, int64_t n_padded, const double* z,
                          const double* N, int64_t count, int32_t num_lines, double* out);
/* log N(y; mu, M M' + diag(d)) (log_mvnpdf_low_rank.m:5-33).  Host buffers, M n x k column-major. */
int gpdla_log_mvnpdf_low_rank_f64(const double* y, const double* mu, const double* M,
                                  const double* d, int64_t n, int32_t k, double* out);

/* ---- GP null-model training objective ----------------------------------------
 * objective.m: f(x) = sum_i spectrum_loss(...) and its gradient g(x), with
 *   x = [M(:) (num_pixels x k, column-major); log_omega (num_pixels); log_c_0; log_tau_0; log_beta]
 * (objective.m:21-30).  The training data are the matrices of learn_qso_model.m:63-84,
 * num_quasars x num_pixels, ROW-major here (row i = quasar i; NaN = missing pixel, objective.m:43).
 * As in the reference, the tau_0 and beta priors enter g only, not f (objective.m:59-71).
 * gpdla_objective_create copies host data to the device (memory = GPDLA_MEM_HOST) or borrows
 * device arrays (GPDLA_MEM_DEVICE, which must outlive the handle); each _eval takes host x and
 * writes host f and g (g may be NULL).  num_pixels <= 4096, k <= 64.  Spectra go through the
 * kernels in launches of up to 2^29 doubles of workspace; the environment variable
 * GPDLA_OBJECTIVE_BATCH (read at create) caps the spectra per launch further. */
typedef struct gpdla_objective gpdla_objective;
int gpdla_objective_create(int32_t device, int64_t num_quasars, int64_t num_pixels, int32_t k,
                           const double* centered_rest_fluxes, const double* lya_1pzs,
                           const double* rest_noise_variances, int32_t memory, gpdla_objective** out);
int gpdla_objective_eval(gpdla_objective* objective, const double* x, double* f, double* g);
void gpdla_objective_destroy(gpdla_objective* objective);
/* spectrum_loss.m:14-76 for one spectrum (host buffers): n pixels, M n x k column-major, omega2
 * per pixel.  Any gradient output may be NULL. */
int gpdla_spectrum_loss_f64(const double* y, const double* lya_1pz, const double* noise_variance,
                            const double* M, const double* omega2, int64_t n, int32_t k, double c_0,
                            double tau_0, double beta, double* nlog_p, double* dM, double* dlog_omega,
                            double* dlog_c_0, double* dlog_tau_0, double* dlog_beta);

/* ---- DLA parameter samples ------------------------------------------------------
 * generate_dla_samples.m:8-57 on the device: the RR2-scrambled Halton points (:8-9), ksdensity of the
 * catalogue's column densities on the 1,000-point fit grid at MATLAB's default bandwidth (:32-33), the
 * quadratic log-density fit (:34, host QR) normalised over [fit_min, fit_upper] (:37-38) and the inverse
 * mixture CDF of every sample's second Halton coordinate (:42-55, fzero), nhi = 10^log_nhi (:57).
 * Host buffers.  The prior's fields are set_parameters.m:49-53's (0.9, 20, 23, 20, 22) and the 25.0 of
 * generate_dla_samples.m:38. */
typedef struct gpdla_dla_prior {
  double alpha;                    /* weight of the fitted component (set_parameters.m:49) */
  double uniform_min, uniform_max; /* uniform component of log10 N_HI (:50-51) */
  double fit_min, fit_max;         /* KDE / fit range (:52-53) */
  double fit_upper;                /* upper limit of the normalising integral (generate_dla_samples.m:38) */
} gpdla_dla_prior;
/* Points start, start + stride, ... (num of them) of the RR2-scrambled Halton sequence in `dims` bases
 * (haltonset(dims, 'Skip', start, 'Leap', stride - 1) + scramble(..., 'RR2'); index 0 is the origin):
 * out[j * dims + d], bit-exact.  Bases 2..64, dims <= 16. */
int gpdla_halton_rr2_f64(int32_t device, int64_t start, int64_t stride, int64_t num, const int32_t* bases,
                         int32_t dims, double* out);
/* log_nhis: the catalogue's n_data column densities (the non-empty cells concatenated, :26-28).
 * Writes num_samples offsets, log10 N_HI and N_HI samples; fit (may be NULL) receives the polyfit
 * coefficients c2, c1, c0, the normaliser Z and the KDE bandwidth.  GPDLA_ENUMERIC when the density
 * estimate vanishes on the fit grid or the fit does not normalise. */
int gpdla_generate_dla_samples_f64(int32_t device, const double* log_nhis, int64_t n_data, int64_t num_samples,
                                   const gpdla_dla_prior* prior, double* offset_samples, double* log_nhi_samples,
                                   double* nhi_samples, double* fit);

/* ---- Spectrum ingest -----------------------------------------------------------
 * read_spec.m:27-38 and preload_qsos.m:18-67 on the device, over the fitsread columns of a catalogue
 * (FITS parsing stays on the host).  Host buffers.  Thresholds are compared exactly (the defaults are
 * all representable in single); brightsky_bit is read_spec.m:9's 1-based bit of the and_mask (24). */
typedef struct gpdla_preload_params {
  double normalization_min_lambda, normalization_max_lambda;   /* set_parameters.m:29-30 (1310, 1325) */
  double min_lambda, max_lambda;                               /* :33-34 (911.75, 1215.75) */
  double loading_min_lambda, loading_max_lambda;               /* :21-22 (910, 1217) */
  int32_t min_num_pixels;                                      /* :26 (200) */
  int32_t brightsky_bit;                                       /* read_spec.m:9 (24) */
} gpdla_preload_params;
/* wavelengths = 10.^loglam (single, correctly rounded), noise_variance = 1 ./ ivar,
 * pixel_mask = ivar == 0 | bitget(and_mask, 24) (read_spec.m:27-38), elementwise over n pixels. */
int gpdla_read_spec_f32(int32_t device, int64_t n, const float* loglam, const float* ivar, const int32_t* and_mask,
                        float* wavelengths, float* noise_variance, uint8_t* pixel_mask);
/* preload_qsos.m:18-67 over num_quasars spectra in CSR (offsets[Q + 1], offsets[0] = 0; the fitsread
 * columns flux, loglam, ivar, and_mask; z_qsos[Q]).  filter_flags[Q] (in/out): entries > 0 are skipped;
 * bit 3 (4) / bit 4 (8) are set for an unnormalisable spectrum / too few pixels.  Out: the cells in CSR
 * (out_offsets[Q + 1]; each out_* array needs offsets[Q] entries at most), normalizers[Q] (0 where not
 * loaded) and, if not NULL, medians[Q] (the single normalisation median, NaN where undefined). */
int gpdla_preload_qsos_f32(int32_t device, int64_t num_quasars, const int64_t* offsets, const float* flux,
                           const float* loglam, const float* ivar, const int32_t* and_mask, const double* z_qsos,
                           const gpdla_preload_params* params, uint8_t* filter_flags, int64_t* out_offsets,
                           float* out_wavelengths, float* out_flux, float* out_noise_variance,
                           uint8_t* out_pixel_mask, double* normalizers, float* medians);

/* Diagnostics (test support; not used by the compute path).
 * Re/Im of the Faddeeva function the line tables are fitted from (host, long double). */
int gpdla_diag_faddeeva_w(double x, double y, double* re, double* im);
/* Max relative error of the fitted profile table of `line` against its long-double source. */
int gpdla_diag_line_table_error(int32_t line, double* max_rel_err);
/* The panel-GEMM weights kernels' raw 3-line absorption exp(-N sum_j lc_j V_j) (before the
 * instrument broadening) at n wavelengths, on the device: f32 = 1 the 24-bit path's packed-fp32
 * profile, f32 = 0 the fp64 one (gemm_i8.hip).  GPDLA_EDEVICE without a device. */
int gpdla_diag_raw_profile3(const double* lambdas, int64_t n, double z, double N, int32_t f32, double* out);

/* Device buffers for callers without a GPU array library (the benchmark, tests, C callers).
 * Callers that already hold device memory (e.g. PyTorch tensors) pass those pointers instead. */
int gpdla_device_malloc(int32_t device, int64_t bytes, void** ptr);
int gpdla_device_free(int32_t device, void* ptr);
int gpdla_memcpy_htod(int32_t device, void* dst, const void* src, int64_t bytes);
int gpdla_memcpy_dtoh(int32_t device, void* dst, const void* src, int64_t bytes);

const char* gpdla_last_error(void);
int32_t gpdla_version(void);
int32_t gpdla_device_count(void);
/* PCI bus id ("dddd:bb:dd.f") of a device, into buf (len >= 13): which physical GPU a rank drives
 * (the multi-GPU bench reports it per rank; process_qsos.m:88's spectra loop split over devices). */
int gpdla_device_pci_bus_id(int32_t device, char* buf, int32_t len);
/* Kernel times (ms, HIP events) of the calling thread's last call of gpdla_read_spec_f32,
 * gpdla_preload_qsos_f32, gpdla_halton_rr2_f64 or gpdla_generate_dla_samples_f64, one per launch in
 * launch order: read_spec 1; preload_qsos 3 (range keys, scan, write); halton 1; generate 3 (KDE,
 * Halton, inverse CDF).  *count = launches recorded (0 for an empty call); at most capacity copied. */
int gpdla_last_call_kernel_ms(double* ms, int32_t capacity, int32_t* count);

#ifdef __cplusplus
}
#endif
#endif /* GPDLA_H */
