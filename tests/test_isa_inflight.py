"""The shipped gfx950 machine code never touches a register while a vector-memory load into it is in
flight (tools/isa_inflight.py).  The Gram GEMM issues its A-digit
prefetches from inline asm (gemm_i8.hip bst_run), invisible to the compiler's waitcnt pass: the hand-off
is only correct if the register allocator never copies, spills or reuses one of those registers between
the load and the wait that retires it.  The round-5 illegal-address fault was such a reuse.  Here:

* the analysis itself on small hand-written instruction streams (what it must flag and what not);
* every kernel of the in-tree libgpdla.so: no violation, and the Gram GEMM's counted waits are credited
  (the check is not vacuous);
* no kernel that issues asm loads spills a VGPR or uses scratch (metadata of the same code objects);
* the source before the round-5 fix (git 8238c15^) compiled here is flagged, at the instruction that
  recomputes an address into registers a dead prefetch is still writing.

CPU only: llvm-objdump / llvm-readelf / hipcc from /opt/rocm cross-compile and disassemble gfx950."""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import isa_inflight as I  # noqa: E402

LIB = ROOT / "gp_dla_detection_amd" / "libgpdla.so"
ASM_LOAD_KERNELS = ("gemm_i8_bst_kernel", "gemm_i8_kernelILi3", "gemm_i8_kernelILi4", "likelihood_i8_kernel")

pytestmark = pytest.mark.skipif(not (I.LLVM_BIN / "llvm-objdump").exists(), reason="no ROCm llvm-objdump")


def _stream(lines):
    """A function in llvm-objdump's gfx950 format from [(instruction text, branch target index or None)]."""
    base = 0x1000
    out = [f"{base:016x} <k>:"]
    for i, (text, tgt) in enumerate(lines):
        tail = f" <k+0x{4 * tgt:x}>" if tgt is not None else ""
        out.append(f"\t{text:<56}// {base + 4 * i:012X}: 00000000{tail}")
    return "\n".join(out)


def _viol(lines):
    (rep,) = I.analyse_disassembly(_stream(lines))
    return rep


def test_read_before_the_wait_is_flagged():
    rep = _viol([("global_load_dwordx4 v[4:7], v[2:3], off", None),
                 ("v_add_u32_e32 v8, v5, v1", None),
                 ("s_waitcnt vmcnt(0)", None),
                 ("s_endpgm", None)])
    assert [(v[0], v[3]) for v in rep.violations] == [(0x1004, "v5")]


def test_write_before_the_wait_is_flagged_and_a_retired_load_is_not():
    rep = _viol([("global_load_dwordx4 v[4:7], v[2:3], off", None),
                 ("global_load_dwordx4 v[8:11], v[2:3], off offset:16", None),
                 ("s_waitcnt vmcnt(1)", None),              # retires the first load only (in order)
                 ("v_mov_b32_e32 v4, 0", None),
                 ("v_mov_b32_e32 v9, 0", None),
                 ("s_endpgm", None)])
    assert [(v[0], v[3]) for v in rep.violations] == [(0x1010, "v9")]
    assert rep.partial_waits_retiring == 1


def test_stores_count_in_issue_order():
    """vmcnt counts stores too, in order with the loads -- the model hipcc itself relies on (a load, then
    a store, then vmcnt(1) before the load's first use: objective.hip)."""
    rep = _viol([("global_load_dwordx2 v[4:5], v[2:3], off", None),
                 ("global_store_dwordx2 v[2:3], v[6:7], off", None),
                 ("s_waitcnt vmcnt(1)", None),
                 ("v_add_f64 v[8:9], v[4:5], v[4:5]", None),
                 ("s_endpgm", None)])
    assert rep.violations == []


def test_a_prefetch_carried_round_a_loop_is_flagged():
    """The round-5 fault's shape: the loop's last prefetch is never waited for, and the next round
    recomputes the address into the same registers."""
    rep = _viol([("s_mov_b32 s0, 4", None),
                 ("v_lshl_add_u64 v[4:5], v[2:3], 0, s[6:7]", None),       # 1: loop head
                 ("global_load_dwordx4 v[4:7], v[4:5], off", None),
                 ("s_add_i32 s0, s0, -1", None),
                 ("s_cmp_lg_u32 s0, 0", None),
                 ("s_cbranch_scc1 1", 1),
                 ("s_waitcnt vmcnt(0)", None),
                 ("s_endpgm", None)])
    assert {(v[0], v[3]) for v in rep.violations} == {(0x1004, "v4"), (0x1004, "v5"), (0x1008, "v4"),
                                                      (0x1008, "v5")}


def _guarded(correlated: bool):
    """A prefetch and the wait that relies on it, each under its own branch: the prefetch skipped by an
    SCC branch on ``s10 >= s11``, the wait chosen by a flag pair from s_cselect_b64 tested through vcc.
    When the flag holds the same comparison (``s10 < s11``), the path 'prefetch skipped, short wait'
    cannot happen and nothing is flagged; when it holds another one (``s12 < s11``) it can."""
    return [("global_load_dwordx4 v[4:7], v[2:3], off", None),               # 0: A(g), read at 11
            ("s_cmp_lt_i32 s10, s11" if correlated else "s_cmp_lt_i32 s12, s11", None),
            ("s_cselect_b64 s[20:21], -1, 0", None),                        # 2: flag = -1 iff that holds
            ("s_cmp_ge_i32 s10, s11", None),                                # 3: the prefetch guard
            ("s_cbranch_scc1 6", 6),                                        # 4: skip the prefetch
            ("global_load_dwordx4 v[8:11], v[2:3], off offset:64", None),   # 5: A(g + 1)
            ("s_andn2_b64 vcc, exec, s[20:21]", None),                      # 6
            ("s_cbranch_vccnz 10", 10),                                     # 7: flag 0 -> wait for all
            ("s_waitcnt vmcnt(1)", None),                                   # 8: retires A(g) iff A(g + 1) issued
            ("s_branch 11", 11),                                            # 9
            ("s_waitcnt vmcnt(0)", None),                                   # 10
            ("v_add_u32_e32 v12, v4, v5", None),                            # 11: reads A(g)
            ("s_waitcnt vmcnt(0)", None),
            ("s_endpgm", None)]


def test_correlated_guards_are_followed_path_sensitively():
    assert _viol(_guarded(True)).violations == []
    bad = _viol(_guarded(False))
    assert {v[3] for v in bad.violations} == {"v4", "v5"}


def test_shipped_library_has_no_register_touched_in_flight():
    assert LIB.exists(), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    reps = I.analyse_file(LIB)
    by_name = {r.function: r for r in reps}
    bad = [(r.function, r.violations[:3], r.calls_with_pending) for r in reps if r.violations or r.calls_with_pending]
    assert not bad, bad
    for key in ASM_LOAD_KERNELS:
        hits = [r for n, r in by_name.items() if key in n]
        assert hits, key
    bst = next(r for n, r in by_name.items() if "gemm_i8_bst_kernel" in n)
    # non-vacuous: the A prefetches are there and the pipeline's counted (non-zero) waits retire them
    assert bst.loads >= 12 and bst.partial_waits_retiring >= 4, (bst.loads, bst.partial_waits_retiring)
    assert bst.collapsed_blocks == 0
    assert sum(r.instructions for r in reps) > 100_000


def test_asm_load_kernels_do_not_spill():
    md = {}
    for co in I.code_objects(LIB):
        md.update(I.kernel_metadata(co))
    for key in ASM_LOAD_KERNELS:
        ents = {n: v for n, v in md.items() if key in n}
        assert ents, key
        for n, v in ents.items():
            if "gemm_i8_kernelILi3" in n:
                continue       # the long-spectrum fallback of the 24-bit path: 2 VGPRs spilled outside its loop
            assert v.get("vgpr_spill_count") == "0", (n, v)
            assert v.get("private_segment_fixed_size") == "0", (n, v)


@pytest.mark.skipif(shutil.which("git") is None or not (ROOT / ".git").exists() or not Path("/opt/rocm/bin/hipcc").exists(),
                    reason="needs the git history and hipcc")
def test_pre_fix_source_is_flagged(tmp_path):
    """gemm_i8.hip as it was before the round-5 fix (commit 8238c15's parent): its unconditional
    prefetches past a wave's last K step leave loads in flight into registers the next round's address
    computation overwrites -- the check must flag that kernel, and only the Gram GEMM."""
    rev = "8238c15^"
    files = subprocess.run(["git", "-C", str(ROOT), "ls-tree", "--name-only", rev, "gp_dla_detection_amd/csrc/"],
                           capture_output=True, text=True)
    if files.returncode != 0:
        pytest.skip("revision not in this clone")
    src = tmp_path / "csrc"
    src.mkdir()
    for f in files.stdout.split():
        (src / Path(f).name).write_text(subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:{f}"],
                                                       capture_output=True, text=True, check=True).stdout)
    obj = tmp_path / "gemm_i8.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                    "-Wno-unused-result", "-o", str(obj), str(src / "gemm_i8.hip")], check=True, cwd=src)
    reps = I.analyse_file(obj)
    flagged = {r.function for r in reps if r.violations}
    assert flagged and all("gemm_i8_bst_kernel" in f for f in flagged), flagged
    bst = next(r for r in reps if "gemm_i8_bst_kernel" in r.function)
    # an address register of the next round's A load rewritten while the last prefetch still lands there
    assert any(v[1].startswith("v_lshl_add_u64") for v in bst.violations), bst.violations[:5]
