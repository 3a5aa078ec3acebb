"""In-flight register check of the gfx950 code objects that ship in libgpdla.so.

A vector-memory load writes its destination VGPRs (or AGPRs) when its data returns, some time after the
instruction issues.  Until an ``s_waitcnt vmcnt(N)`` retires it, no instruction may read those registers
(it would see stale data) or write them (the returning load would overwrite the value).  The compiler's
waitcnt pass guarantees this for the loads it generates; for loads issued from inline asm (the Gram
GEMM's A-digit prefetches, ``gemm_i8.hip`` ``bst_run``: ``load_a`` / ``land``) it sees nothing, and the
hand-off rests on the register allocator never copying, spilling or reusing a register between the
asm load and its wait.  The round-5 illegal-address fault (``profiles/round5/ab/r10g``) came from exactly
such a reuse: prefetches past a wave's last K step left registers the compiler considered dead while the
hardware could still write them.  This module checks the property on the SHIPPED machine code:

1. the ``.hip_fatbin`` section of the library (or of a ``hipcc -c`` object) is split into its clang
   offload bundles and the gfx950 code object of each translation unit is taken out;
2. ``llvm-objdump -d --mcpu=gfx950`` disassembles it;
3. a forward data-flow analysis over each kernel's control-flow graph tracks every pending load's
   destination registers with the number of vector-memory operations issued after it (its "age");
   ``s_waitcnt vmcnt(N)`` retires a load whose age is >= N.  Loads, stores, atomics and LDS-DMA all count,
   in issue order: the model the compiler itself relies on for gfx950 (e.g. objective.hip's
   ``global_load_dwordx2`` ... ``global_store_dwordx2`` ... ``s_waitcnt vmcnt(1)`` before the load's first
   use).  At a join a register stays pending with its smallest age (the least-retired path).
4. Any instruction that names a pending register -- as a source or as a destination -- is a violation,
   except a newer load writing the same register (loads return in order, the newer value lands last).

Path sensitivity.  The code that guards a prefetch and the code that guards its consumer test the same
scalar condition, but the compiler materialises it in different forms: an ``s_cmp`` feeding an
``s_cbranch_scc*`` in one place, the same comparison kept as a 0 / -1 SGPR pair (``s_cselect_b64`` or
``s_mov_b64``) and tested later with ``s_and(n2)_b64 vcc, exec, s[..]`` + ``s_cbranch_vcc(n)z``.  A
path-insensitive analysis would follow "prefetch issued, consumer skipped" paths the program cannot
take.  So each state also carries a small environment of scalar facts: the comparison an SCC value or a
flag pair holds (a comparison instance is identified by its instruction and lives while none of its
operand SGPRs is written), and the outcomes of the branches taken on this path.  A branch whose outcome
the facts decide has one successor.  Everything that may write an SGPR, SCC or vcc forgets what it held
(VALU instructions forget every SGPR they name), so facts are only ever lost, never invented; an
environment is dropped at a block that collects too many (ENV_CAP), which is sound too.  One assumption:
exec != 0 where a flag pair is tested (the tests are uniform branches).

    python tools/isa_inflight.py [libgpdla.so | object.o ...]      report per kernel, exit 1 on a violation
"""
from __future__ import annotations

import re
import struct
import subprocess
import sys
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

LLVM_BIN = Path("/opt/rocm/lib/llvm/bin")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
AGE_CAP = 64    # vmcnt is a 6-bit field on gfx9: an age of 64 is retired by any wait
ENV_CAP = 64    # scalar-fact environments kept apart per block before they are dropped there

_REG_RANGE = re.compile(r"(?<![\w\]])([va])\[(\d+):(\d+)\]")
_REG_ONE = re.compile(r"(?<![\w\]])([va])(\d+)(?![\w\[])")
_SREG_RANGE = re.compile(r"(?<![\w\]])s\[(\d+):(\d+)\]")
_SREG_ONE = re.compile(r"(?<![\w\]])s(\d+)(?![\w\[])")
_TARGET = re.compile(r"<([^>+]+)(?:\+0x([0-9a-fA-F]+))?>")
_FUNC = re.compile(r"^([0-9a-fA-F]+) <([^>]+)>:$")
_INSN = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")
_FLAG_DEF = re.compile(r"s\[(\d+):(\d+)\],\s*(0|-1)")
_FLAG_SEL = re.compile(r"s\[(\d+):(\d+)\],\s*(0|-1),\s*(0|-1)")
_FLAG_TEST = re.compile(r"vcc,\s*exec,\s*s\[(\d+):(\d+)\]")
_CMP = re.compile(r"s_cmp_(eq|lg|gt|ge|lt|le)_(i32|u32|u64)")

VMEM_PREFIXES = ("global_", "buffer_", "flat_", "scratch_", "tbuffer_")
VMCNT_KINDS = ("load", "lds_dma", "store", "atomic_ret")   # the instructions that count on vmcnt
# scalar instructions with no SGPR destination (the first operand of every other SALU op is its SDST)
_NO_SDST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_barrier", "s_setprio",
            "s_sleep", "s_sendmsg", "s_endpgm", "s_trap", "s_icache", "s_setreg", "s_set_gpr_idx", "s_ttrace",
            "s_setkill", "s_incperflevel", "s_decperflevel", "s_denorm_mode", "s_round_mode", "s_setvskip")
# scalar instructions that leave SCC alone
_KEEP_SCC = ("s_mov_", "s_movk_", "s_cselect_", "s_cmov", "s_waitcnt", "s_nop", "s_barrier", "s_setprio",
             "s_sleep", "s_cbranch", "s_branch", "s_getpc", "s_load", "s_buffer_load", "s_sendmsg", "s_set_gpr_idx")


# ---------------------------------------------------------------------------------------------- extraction
def code_objects(path: Path) -> list[bytes]:
    """The gfx950 code objects in ``path``'s .hip_fatbin section (one clang offload bundle per TU)."""
    with tempfile.TemporaryDirectory() as td:
        sec = Path(td) / "fatbin.bin"
        subprocess.run([str(LLVM_BIN / "llvm-objcopy"), f"--dump-section=.hip_fatbin={sec}", str(path),
                        str(Path(td) / "x")], check=True, capture_output=True)
        data = sec.read_bytes()
    out = []
    pos = data.find(BUNDLE_MAGIC)
    while pos != -1:
        q = pos + len(BUNDLE_MAGIC)
        (n,) = struct.unpack_from("<Q", data, q)
        q += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            q += 24
            triple = data[q:q + tlen].decode()
            q += tlen
            if triple.endswith("gfx950") and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(BUNDLE_MAGIC, pos + 1)
    return out


def kernel_metadata(co: bytes) -> dict:
    """{kernel symbol: {field: value}} from the code object's AMDGPU metadata note (.vgpr_count,
    .vgpr_spill_count, .private_segment_fixed_size, ...)."""
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        r = subprocess.run([str(LLVM_BIN / "llvm-readelf"), "--notes", f.name], check=True, capture_output=True,
                           text=True)
    out, cur = {}, {}
    for line in r.stdout.splitlines():
        m = re.match(r"^  (- |  )\.([a-z_]+):\s+(\S+)\s*$", line)   # kernel-level fields only (args nest deeper)
        if not m:
            continue
        if m.group(1) == "- ":       # a new kernel entry
            cur = {}
        cur[m.group(2)] = m.group(3)
        if m.group(2) == "name":
            out[m.group(3)] = cur
    return out


def disassemble(co: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        r = subprocess.run([str(LLVM_BIN / "llvm-objdump"), "-d", "--mcpu=gfx950", f.name],
                           check=True, capture_output=True, text=True)
    return r.stdout


# ---------------------------------------------------------------------------------------------- parsing
def regs_in(text: str) -> set:
    """VGPRs / AGPRs named in an operand string, as ('v'|'a', index)."""
    out = set()
    for k, lo, hi in _REG_RANGE.findall(text):
        out.update((k, i) for i in range(int(lo), int(hi) + 1))
    for k, i in _REG_ONE.findall(_REG_RANGE.sub(" ", text)):
        out.add((k, int(i)))
    return out


def sregs_in(text: str) -> set:
    out = set()
    for lo, hi in _SREG_RANGE.findall(text):
        out.update(range(int(lo), int(hi) + 1))
    out.update(int(i) for i in _SREG_ONE.findall(_SREG_RANGE.sub(" ", text)))
    return out


def split_operands(ops: str) -> list[str]:
    parts, depth, cur = [], 0, ""
    for ch in ops:
        if ch in "[(":
            depth += 1
        elif ch in "])":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return parts


@dataclass
class Insn:
    addr: int
    mnem: str
    ops: str
    kind: str = "other"          # load | lds_dma | store | atomic_ret | wait | branch | cbranch | end | call | other
    dst: set = field(default_factory=set)
    src: set = field(default_factory=set)
    vmcnt: int | None = None
    target: int | None = None
    # scalar side (path facts)
    swrites: frozenset = frozenset()   # SGPRs this instruction may write
    kills_all_sgprs: bool = False      # indirect SGPR writes (s_movreld)
    writes_scc: bool = False
    mentions_vcc: bool = False
    cmp: tuple | None = None           # s_cmp: (canonical key, operand SGPRs, polarity)
    flag_def: tuple | None = None      # s_mov_b64 s[lo:hi], 0 | -1                    -> (lo, hi, value)
    flag_sel: tuple | None = None      # s_cselect_b64 s[lo:hi], -1, 0 (or 0, -1)       -> (lo, hi, SCC=1 gives -1)
    flag_test: tuple | None = None     # s_and(n2)_b64 vcc, exec, s[lo:hi]               -> (lo, hi, is_andn2)


def _canon_cmp(op: str, ty: str, a: str, b: str):
    """s_cmp_<op>_<ty> a, b -> (key, polarity): the comparison is true iff predicate ``key`` == polarity."""
    if op == "lt":
        return ("lt", ty, a, b), True
    if op == "ge":
        return ("lt", ty, a, b), False
    if op == "gt":
        return ("lt", ty, b, a), True
    if op == "le":
        return ("lt", ty, b, a), False
    x, y = sorted((a, b))
    return ("eq", ty, x, y), op == "eq"


def classify(addr: int, mnem: str, ops: str, tail: str, func_addr: dict) -> Insn:
    ins = Insn(addr, mnem, ops.strip())
    body = ins.ops
    ins.mentions_vcc = bool(re.search(r"\bvcc(_lo|_hi)?\b", body))
    if mnem.startswith("s_"):
        parts = split_operands(body)
        if not mnem.startswith(_NO_SDST) and parts:
            ins.swrites = frozenset(sregs_in(parts[0]))
        ins.kills_all_sgprs = mnem.startswith("s_movreld")
        ins.writes_scc = not mnem.startswith(_KEEP_SCC)
        m = _CMP.fullmatch(mnem)
        if m and len(parts) == 2:
            key, pol = _canon_cmp(m.group(1), m.group(2), parts[0], parts[1])
            ins.cmp = (key, frozenset(sregs_in(body)), pol)
        m = _FLAG_DEF.fullmatch(body)
        if mnem == "s_mov_b64" and m:
            ins.flag_def = (int(m.group(1)), int(m.group(2)), int(m.group(3)))
        m = _FLAG_SEL.fullmatch(body)
        if mnem == "s_cselect_b64" and m and {m.group(3), m.group(4)} == {"0", "-1"}:
            ins.flag_sel = (int(m.group(1)), int(m.group(2)), m.group(3) == "-1")
        m = _FLAG_TEST.fullmatch(body)
        if mnem in ("s_andn2_b64", "s_and_b64") and m:
            ins.flag_test = (int(m.group(1)), int(m.group(2)), mnem == "s_andn2_b64")
    else:
        ins.swrites = frozenset(sregs_in(body))     # VALU: any SGPR named may be a destination (v_cmp, carry-out)
    if mnem.startswith(VMEM_PREFIXES):
        toks = body.replace(",", " ").split()
        if "_lds_" in mnem or "lds" in toks:
            ins.kind, ins.src = "lds_dma", regs_in(body)
        elif "_load" in mnem:
            parts = split_operands(body)
            ins.kind, ins.dst = "load", regs_in(parts[0]) if parts else set()
            ins.src = regs_in(", ".join(parts[1:]))
        elif "_atomic" in mnem and "sc0" in toks:
            parts = split_operands(body)
            ins.kind, ins.dst = "atomic_ret", regs_in(parts[0]) if parts else set()
            ins.src = regs_in(", ".join(parts[1:]))
        elif "_store" in mnem or "_atomic" in mnem:
            ins.kind, ins.src = "store", regs_in(body)
        else:                    # cache maintenance (buffer_wbl2, buffer_inv, ...): no registers, no count
            ins.kind, ins.src = "other", regs_in(body)
        return ins
    if mnem == "s_waitcnt":
        ins.kind = "wait"
        m = _VMCNT.search(body)
        if m:
            ins.vmcnt = int(m.group(1))
        elif re.fullmatch(r"\s*(0x[0-9a-fA-F]+|\d+)\s*", body):
            simm = int(body.strip(), 0)
            ins.vmcnt = (simm & 0xF) | ((simm >> 14) & 0x3) << 4
        return ins
    if mnem == "s_endpgm":
        ins.kind = "end"
        return ins
    if mnem in ("s_setpc_b64", "s_swappc_b64"):
        ins.kind = "call"
        return ins
    if mnem == "s_branch" or mnem.startswith("s_cbranch_"):
        m = _TARGET.search(tail)
        if m is None:
            raise ValueError(f"branch without a resolved target at {addr:#x}: {mnem} {body}")
        ins.target = func_addr[m.group(1)] + (int(m.group(2), 16) if m.group(2) else 0)
        ins.kind = "branch" if mnem == "s_branch" else "cbranch"
        return ins
    if mnem.startswith("s_"):
        return ins               # scalar instructions name no vector registers
    ins.src = regs_in(body)      # VALU / MFMA / LDS / DPP: every register named is accessed
    return ins


def parse(disasm: str) -> dict:
    """{function name: [Insn ...]} in address order."""
    func_addr = {}
    for line in disasm.splitlines():
        m = _FUNC.match(line)
        if m:
            func_addr[m.group(2)] = int(m.group(1), 16)
    funcs, cur = {}, None
    for line in disasm.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = funcs.setdefault(m.group(2), [])
            continue
        m = _INSN.match(line)
        if m and cur is not None:
            cur.append(classify(int(m.group(3), 16), m.group(1), m.group(2), m.group(4), func_addr))
    return funcs


# ---------------------------------------------------------------------------------------------- analysis
@dataclass
class Report:
    function: str
    instructions: int
    loads: int
    partial_waits_retiring: int  # waits vmcnt(N > 0) that retire at least one pending load
    violations: list             # (insn addr, mnemonic, operands, register, load addr)
    calls_with_pending: list
    path_states: int = 0         # (block, scalar environment) pairs the analysis visited
    collapsed_blocks: int = 0    # blocks where environments were dropped (ENV_CAP)


def _transfer(ins: Insn, st: dict, viol: list | None, stats: dict | None):
    """Apply one instruction to the pending state {reg: (age, load addr)} (in place)."""
    k = ins.kind
    if k == "wait":
        if ins.vmcnt is not None:
            dead = [r for r, (age, _) in st.items() if age >= ins.vmcnt]
            if stats is not None and dead and ins.vmcnt > 0:
                stats["partial"].add(ins.addr)
            for r in dead:
                del st[r]
        return
    touched = ins.src if k in ("load", "atomic_ret") else ins.src | ins.dst
    if viol is not None:
        for r in touched & st.keys():
            viol.append((ins.addr, ins.mnem, ins.ops, f"{r[0]}{r[1]}", st[r][1]))
    if k in VMCNT_KINDS:
        for r, (age, a) in list(st.items()):
            st[r] = (min(age + 1, AGE_CAP), a)
    if k in ("load", "atomic_ret"):
        for r in ins.dst:
            st[r] = (0, ins.addr)


# Scalar environment entries (a frozenset of tuples):
#   ("s", lo, hi, v)          s[lo:hi] holds the constant v (0 or -1)
#   ("sb", lo, hi, p, pol)    s[lo:hi] is -1 iff predicate p == pol, else 0
#   ("scc", p, pol)           SCC is 1 iff p == pol
#   ("vcc", nz)               vcc != 0 is known
#   ("vccp", p, pol)          vcc != 0 iff p == pol
#   ("pred", p, key, regs)    p (the address of the s_cmp that created it) still equals comparison ``key``
#                             of the current values of ``regs`` (none written since)
#   ("fact", p, val)          on this path p == val
def _refs(e):
    return e[3] if e[0] == "sb" else e[1] if e[0] in ("scc", "vccp", "pred", "fact") else None


def _prune(env: set) -> frozenset:
    live = {_refs(e) for e in env if e[0] != "fact"}
    return frozenset(e for e in env if e[0] != "fact" or e[1] in live)


def _edge(env) -> frozenset:
    """The environment carried along a CFG edge: comparison instances are only kept for common-
    subexpression matching inside a block, and a branch outcome only while a flag, SCC or vcc still
    holds that comparison (which keeps the number of environments per block small)."""
    e = {x for x in env if x[0] != "pred"}
    live = {_refs(x) for x in e if x[0] != "fact"}
    return frozenset(x for x in e if x[0] != "fact" or x[1] in live)


def _env_step(ins: Insn, env: frozenset) -> frozenset:
    if not env and ins.cmp is None and ins.flag_def is None:
        return env
    e = set(env)
    scc = next((x for x in e if x[0] == "scc"), None)
    # reads first
    new = []
    if ins.cmp is not None:
        key, regs, pol = ins.cmp
        p = next((x[1] for x in e if x[0] == "pred" and x[2] == key), None)
        if p is None:                          # a new instance: what referred to an old one is stale
            p = ins.addr
            e = {x for x in e if _refs(x) != p}
            new.append(("pred", p, key, regs))
        new.append(("scc", p, pol))
    if ins.flag_sel is not None and scc is not None:
        lo, hi, one_gives_m1 = ins.flag_sel
        new.append(("sb", lo, hi, scc[1], scc[2] if one_gives_m1 else not scc[2]))
    if ins.flag_def is not None:
        new.append(("s",) + ins.flag_def)
    if ins.flag_test is not None:
        lo, hi, andn2 = ins.flag_test
        for x in e:
            if x[0] == "s" and (x[1], x[2]) == (lo, hi):
                new.append(("vcc", (x[3] == 0) if andn2 else (x[3] == -1)))   # vcc = exec & ~s  or  exec & s
            elif x[0] == "sb" and (x[1], x[2]) == (lo, hi):
                new.append(("vccp", x[3], (not x[4]) if andn2 else x[4]))
    # then writes
    if ins.kills_all_sgprs:
        e = {x for x in e if x[0] not in ("s", "sb", "pred")}
    if ins.swrites:
        w = ins.swrites
        e = {x for x in e if not ((x[0] in ("s", "sb") and any(x[1] <= r <= x[2] for r in w))
                                  or (x[0] == "pred" and x[3] & w))}
    if ins.writes_scc or ins.cmp is not None:
        e = {x for x in e if x[0] != "scc"}
    if ins.mentions_vcc:
        e = {x for x in e if x[0] not in ("vcc", "vccp")}
    e.update(new)
    return _prune(e)


def _merge(a: dict | None, b: dict) -> dict:
    if a is None:
        return dict(b)
    out = dict(a)
    for r, v in b.items():
        if r not in out or v[0] < out[r][0]:
            out[r] = v
    return out


def analyse_function(name: str, insns: list) -> Report:
    if not insns:
        return Report(name, 0, 0, 0, [], [])
    index = {ins.addr: i for i, ins in enumerate(insns)}
    # basic blocks: leaders = entry, branch targets, instructions after a branch / end
    leaders = {0}
    for i, ins in enumerate(insns):
        if ins.kind in ("branch", "cbranch", "end", "call"):
            if i + 1 < len(insns):
                leaders.add(i + 1)
            if ins.target is not None:
                if ins.target not in index:
                    raise ValueError(f"{name}: branch target {ins.target:#x} is not an instruction")
                leaders.add(index[ins.target])
    starts = sorted(leaders)
    bounds = {s: (starts[j + 1] if j + 1 < len(starts) else len(insns)) for j, s in enumerate(starts)}

    def succ(s, env):
        """[(successor block, environment on that edge)]"""
        last = insns[bounds[s] - 1]
        nxt = bounds[s] if bounds[s] < len(insns) else None
        env = _edge(env)
        if last.kind in ("end", "call"):
            return []
        if last.kind == "branch":
            return [(index[last.target], env)]
        if last.kind != "cbranch":
            return [(nxt, env)] if nxt is not None else []
        tgt = index[last.target]
        both = [(tgt, env)] + ([(nxt, env)] if nxt is not None else [])
        m = last.mnem
        if m in ("s_cbranch_vccnz", "s_cbranch_vccz"):
            known = next((x for x in env if x[0] in ("vcc", "vccp")), None)
            if known is None:
                return both
            if known[0] == "vcc":
                taken = known[1] == (m == "s_cbranch_vccnz")
                return [(tgt, env)] if taken else ([(nxt, env)] if nxt is not None else [])
            p, pol_nz = known[1], known[2]                 # vcc != 0 iff p == pol_nz
            pol_taken = pol_nz if m == "s_cbranch_vccnz" else not pol_nz
        elif m in ("s_cbranch_scc1", "s_cbranch_scc0"):
            known = next((x for x in env if x[0] == "scc"), None)
            if known is None:
                return both
            p, pol_one = known[1], known[2]                # SCC == 1 iff p == pol_one
            pol_taken = pol_one if m == "s_cbranch_scc1" else not pol_one
        else:
            return both
        fact = next((x[2] for x in env if x[0] == "fact" and x[1] == p), None)
        if fact is not None:
            taken = fact == pol_taken
            return [(tgt, env)] if taken else ([(nxt, env)] if nxt is not None else [])
        out = [(tgt, _edge(set(env) | {("fact", p, pol_taken)}))]
        if nxt is not None:
            out.append((nxt, _edge(set(env) | {("fact", p, not pol_taken)})))
        return out

    def run_block(key, pending, viol=None, stats=None, calls=None):
        s, env = key
        st = dict(pending)
        for i in range(s, bounds[s]):
            ins = insns[i]
            if calls is not None and ins.kind == "call" and st:
                calls.append((ins.addr, ins.mnem, sorted(st)))
            _transfer(ins, st, viol, stats)
            env = _env_step(ins, env)
        return st, env

    empty = frozenset()
    state_in = {(0, empty): {}}
    envs_at = {0: {empty}}
    collapsed = set()
    work = [(0, empty)]
    while work:
        key = work.pop()
        if key not in state_in:
            continue
        st, env = run_block(key, state_in[key])
        for t, env_t in succ(key[0], env):
            if t in collapsed:
                env_t = empty
            elif env_t not in envs_at.setdefault(t, set()):
                envs_at[t].add(env_t)
                if len(envs_at[t]) > ENV_CAP:     # too many: drop the scalar facts at this block
                    collapsed.add(t)
                    acc = None
                    for e in envs_at.pop(t):
                        if (t, e) in state_in:
                            acc = _merge(acc, state_in.pop((t, e)))
                    state_in[(t, empty)] = _merge(acc, st) if acc is not None else dict(st)
                    work.append((t, empty))
                    continue
            tkey = (t, env_t)
            merged = _merge(state_in.get(tkey), st)
            if merged != state_in.get(tkey):
                state_in[tkey] = merged
                work.append(tkey)
    viol, stats, calls = [], {"partial": set()}, []
    for key, pending in state_in.items():
        run_block(key, pending, viol, stats, calls)
    seen, uniq = set(), []
    for v in sorted(viol):
        if (v[0], v[3]) not in seen:
            seen.add((v[0], v[3]))
            uniq.append(v)
    loads = sum(1 for ins in insns if ins.kind == "load")
    return Report(name, len(insns), loads, len(stats["partial"]), uniq, calls, len(state_in), len(collapsed))


def analyse_disassembly(disasm: str) -> list:
    return [analyse_function(n, ins) for n, ins in parse(disasm).items()]


def analyse_file(path: Path) -> list:
    return [r for co in code_objects(path) for r in analyse_disassembly(disassemble(co))]


def demangle(names: list) -> list:
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main(argv: list) -> int:
    root = Path(__file__).resolve().parents[1]
    paths = [Path(p) for p in argv] or [root / "gp_dla_detection_amd" / "libgpdla.so"]
    bad = 0
    for p in paths:
        reps = analyse_file(p)
        names = demangle([r.function for r in reps])
        print(f"# {p}: {len(reps)} functions, {sum(r.instructions for r in reps)} instructions, "
              f"{sum(r.loads for r in reps)} register loads")
        for r, n in zip(reps, names):
            flag = "VIOLATION" if r.violations or r.calls_with_pending else "ok"
            print(f"{flag:9s} {n}: {r.instructions} insns, {r.loads} loads, {r.partial_waits_retiring} partial vmcnt "
                  f"waits retiring loads, {r.path_states} path states, {r.collapsed_blocks} collapsed blocks, "
                  f"{len(r.violations)} violations")
            for v in r.violations[:20]:
                print(f"    {v[0]:#x} {v[1]} {v[2]}  <- {v[3]} still in flight from the load at {v[4]:#x}")
            bad += len(r.violations) + len(r.calls_with_pending)
    print("violations:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
