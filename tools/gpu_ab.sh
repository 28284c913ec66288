# The one A/B script: interleaved runs of bench.py under several variants.
#   bash tools/gpu_ab.sh [--tests "<pytest files>"] [--rounds N] <workload> <variant>...
# workload: headline | repair128 | repair512 | repair512q3 | split512 | mixed, or
#           "bench:<bench.py args>" for anything else
# variant:  label=VAR=v,VAR=v   environment settings (label= alone: defaults),
#           label=lib:<path>    another build of libdagpu.so (DAGPU_LIB), or
#           label=args:<args>   extra bench.py arguments
# Prints one line per run: label, value, ms per step, bit-exact flag.
set -o pipefail
mkdir -p gpurun_out
tests=""; rounds=2
while [ $# -gt 0 ]; do
  case $1 in
    --tests) tests=$2; shift 2;;
    --rounds) rounds=$2; shift 2;;
    *) break;;
  esac
done
wl=$1; shift
case $wl in
  headline) args="--steps 20 --warmup 3 --no-cpu --no-replay --no-e2e --no-configs";;
  repair128) args="--mode repair --k 128 --batch 256 --steps 5 --warmup 1";;
  repair512) args="--mode repair --k 512 --batch 2 --steps 5 --warmup 1";;
  repair512q3) args="--mode repair --k 512 --batch 2 --steps 5 --warmup 1 --pattern q3";;
  split512) args="--mode split --split-k 512 --steps 5 --warmup 1";;
  mixed) args="--mode mixed --steps 3 --warmup 1";;
  bench:*) args=${wl#bench:};;
  *) echo "unknown workload $wl"; exit 2;;
esac
if [ -n "$tests" ]; then
  timeout -k 10 600 python -u -m pytest $tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    label=${spec%%=*}; rest=${spec#*=}
    envs=(); extra=""; unset DAGPU_LIB
    if [ "${rest#lib:}" != "$rest" ]; then export DAGPU_LIB=${rest#lib:};
    elif [ "${rest#args:}" != "$rest" ]; then extra=${rest#args:};
    elif [ -n "$rest" ]; then IFS=, read -ra envs <<< "$rest"; fi
    log=gpurun_out/ab_${label}_$r.log
    env "${envs[@]}" timeout -k 10 300 python -u bench.py $args $extra > $log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 $log; exit $rc; fi
    python3 - "$label" "$log" <<'PY'
import json, sys
label, log = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(log) if l.startswith('{"metric"')][-1])
ok = d.get("headline_bit_exact", d.get("bit_exact"))
print(f"{label}: {d['value']:.1f} {d['unit']}, {d['ms_per_step']:.3f} ms/step, bit_exact {ok}")
PY
  done
done
unset DAGPU_LIB
