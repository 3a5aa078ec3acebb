#!/bin/bash
# One GPU-box session, parametrised (replaces the per-session gpu_r*.sh scripts of rounds 1-2; their
# records stay under profiles/).  Every step runs under its own time limit; the first failing step
# ends the session (no GPU step after a fault, abort or timeout).
#
#   tools/gpu_run.sh <tag> <step> [<step> ...]        outputs under gpurun_out/<tag>/
#
# steps:
#   tests[=<pytest -k expr>]     the -m gpu suite (or the tests matching the expression)
#   testfile=<path>              one test file (-m gpu)
#   smoke                        __graft_entry__.smoke()
#   py=<script>[=<args>]         python <script> <args>            -> <script name>.log
#   bench=<name>[=<args>]        python bench.py <args>            -> <name>.json
#   dist=<N>=<name>[=<args>]     torchrun, N ranks sharing the leased GPU -> <name>.json
#   prof=<name>[=<args>]         tools/profile.sh <tag>_<name> <args> (trace, FETCH, WRITE, SQ)
#   stall=<name>[=<args>]        tools/profile_stalls.sh <tag>_<name> <args> (issue / wait / MFMA-busy counters)
#   lib=<variant.so>             GPDLA_LIB for the following steps (A/B variants; "head" = in-tree)
#   ab=<reps>=<v1,v2,..>[=<args>]  interleaved bench A/B over tools/variants/<v>.so (head = in-tree)
set -uo pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
PORT=29600
summ() {  # one-line summary of a bench JSON line
  python3 - "$1" <<'EOF'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
except Exception as e:
    print("  (no JSON)", e); sys.exit(0)
r = d.get("roofline", {})
print(f"  value {d.get('value', 0):.4g} {d.get('unit', '')}  ms/step {d.get('ms_per_step', 0):.2f}  n_gpus {d.get('n_gpus')}"
      f"  kernel {d.get('kernel_ms', {}).get('likelihood', 'n/a')}  frac {r.get('frac', 'n/a')}  ok {d.get('checks_ok', 'n/a')}"
      + (f"  e2e {d['e2e']}" if 'e2e' in d else ""))
EOF
}
run() {  # run <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$log" 2> "${log%.*}.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; tail -20 "${log%.*}.err"; tail -20 "$log"; exit $rc; fi
}
for step in "$@"; do
  IFS='=' read -r kind a b c <<< "$step"
  echo "== $step"
  case "$kind" in
    tests)
      if [ -n "${a:-}" ]; then K=(-k "$a"); else K=(); fi
      run 1100 "$O/gpu_tests.log" python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread "${K[@]}"
      tail -1 "$O/gpu_tests.log" ;;
    testfile)
      run 1100 "$O/$(basename "$a" .py).log" python -u -m pytest "$a" -m gpu -v -s --timeout 900 --timeout-method thread
      tail -1 "$O/$(basename "$a" .py).log" ;;
    py)
      run 600 "$O/$(basename "$a" .py).log" python "$a" ${b:-}
      tail -40 "$O/$(basename "$a" .py).log" ;;
    smoke)
      run 300 "$O/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
      tail -1 "$O/smoke.log" ;;
    bench)
      run 900 "$O/$a.json" python bench.py ${b:-}
      summ "$O/$a.json" ;;
    dist)
      PORT=$((PORT + 1))
      run 1100 "$O/$b.json" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$a" --master-addr 127.0.0.1 \
          --master-port $PORT bench.py --gpus "$a" ${c:-}
      summ "$O/$b.json" ;;
    prof)
      run 1100 "$O/prof_$a.log" bash tools/profile.sh "${TAG}_$a" ${b:-}
      tail -1 "$O/prof_$a.log" ;;
    stall)
      run 1100 "$O/stall_$a.log" bash tools/profile_stalls.sh "${TAG}_$a" ${b:-}
      tail -1 "$O/stall_$a.log" ;;
    lib)
      if [ "$a" = head ]; then unset GPDLA_LIB; else export GPDLA_LIB=$PWD/$a; fi ;;
    ab)
      for r in $(seq 1 "$a"); do
        for v in ${b//,/ }; do
          if [ "$v" = head ]; then L=""; else L=$PWD/tools/variants/$v.so; fi
          GPDLA_LIB=$L run 600 "$O/ab_${v}_$r.json" python bench.py --cpu-budget 0 --no-alt ${c:-}
          echo -n "$v $r"; summ "$O/ab_${v}_$r.json"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo all-done
