#!/bin/bash
# One gpurun call = one list of named steps, each under its own time limit,
# stopping at the first failure (a fault, abort or timeout ends the call).
#
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh <out> <step> [<step> ...]
#
# Output lands in gpurun_out/<out>/<step>.{json,log,err}.  Steps:
#   tests             full GPU suite (pytest -m gpu)
#   smoke             __graft_entry__.smoke()
#   bench             the driver's default command (bench.py --steps 20 --warmup 5)
#   bench_c3|bench_c4 bench.py --config c3|c4 (single config)
#   simN              emulated rank 0 of an N-GPU job (bench.py --sim-world N --no-cpu)
#   prof_c2|prof_c3|prof_c4|prof_simN
#                     rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes
#                     (tools/profile_round.sh) of the headline plan of that shape
#   prof:<cfg>:<fmt>  the same for ONE format of config <cfg> (c2|c3|c4)
#   rehearsal8        bench.py --gpus 8 at the config-5 shape, 8 gloo ranks on one GPU
#   gloo2_c3          the self-launched 2-rank bench (gloo, one GPU) with --verify
#   pt:<selection>    pytest -m gpu on the named tests only ("tests/x.py::test_a tests/y.py")
#   py:<script args>  python3 -u <script args> (a tools/ probe), stdout to <step>.log
#   exe:<binary args>  a stand-alone probe binary (bin/region_probe ...)
#   probe:<script args> the same against the probe build (make probes:
#                     SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so)
# This replaces round 2's one-off tools/r2_*.sh wrappers (profiles/round2/README.md).
set -o pipefail
OUTNAME=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$OUTNAME
mkdir -p "$O"
cd "$R"
export PYTHONUNBUFFERED=1
i=0
for step in "$@"; do
  i=$((i + 1))
  tag=$(printf '%02d_%s' $i "$(printf "%s" "$step" | tr -c 'A-Za-z0-9_.-' '_' | cut -c1-40)")
  echo "[$(date +%T)] step $tag" >&2
  case "$step" in
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          > "$O/$tag.log" 2>&1 ;;
    smoke)
      timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/$tag.log" 2>&1 ;;
    bench)
      timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > "$O/$tag.json" 2> "$O/$tag.err" ;;
    bench_c3|bench_c4)
      timeout -k 10 400 python3 -u bench.py --config "${step#bench_}" --only-config > "$O/$tag.json" 2> "$O/$tag.err" ;;
    sim[0-9]*)
      timeout -k 10 400 python3 -u bench.py --sim-world "${step#sim}" --no-cpu --only-config \
          > "$O/$tag.json" 2> "$O/$tag.err" ;;
    prof_c2|prof_c3|prof_c4)
      timeout -k 10 1000 bash tools/profile_round.sh "${OUTNAME}_${step#prof_}" --config "${step#prof_}" \
          --formats auto --only-config --steps 20 --warmup 5 --trials 3 > "$O/$tag.log" 2>&1 ;;
    prof_sim[0-9]*)
      timeout -k 10 1000 bash tools/profile_round.sh "${OUTNAME}_${step#prof_}" --sim-world "${step#prof_sim}" \
          --formats auto --only-config --steps 20 --warmup 5 --trials 3 > "$O/$tag.log" 2>&1 ;;
    prof:*)
      # prof:<config>:<format>: one format of one config per profile (PMC keys
      # name the kernels of one execute, tools/pmc_summary.py)
      spec=${step#prof:}; cfg=${spec%%:*}; fmt=${spec#*:}
      timeout -k 10 1000 bash tools/profile_round.sh "${OUTNAME}_${cfg}_${fmt}" --config "$cfg" \
          --formats "$fmt" --only-config --steps 20 --warmup 5 --trials 3 > "$O/$tag.log" 2>&1 ;;
    rehearsal8)
      # the 8-rank flow at the config-5 shape on ONE GPU (gloo: the ranks share
      # the device; kernel times are meaningless, setup time / memory are not)
      BENCH_DIST_BACKEND=gloo timeout -k 10 1100 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 --trials 1 \
          > "$O/$tag.json" 2> "$O/$tag.err" ;;
    gloo2_c3)
      BENCH_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 2 --config c3 --rows 500000 \
          --formats auto --no-cpu --only-config --verify > "$O/$tag.json" 2> "$O/$tag.err" ;;
    pt:*)
      # pt:<pytest selection>: named GPU tests only
      # shellcheck disable=SC2086
      timeout -k 10 900 python3 -u -m pytest ${step#pt:} -m gpu -x -v -s --timeout 600 --timeout-method thread \
          > "$O/$tag.log" 2>&1 ;;
    py:*)
      # shellcheck disable=SC2086
      timeout -k 10 600 python3 -u ${step#py:} > "$O/$tag.log" 2> "$O/$tag.err" ;;
    probe:*)
      # shellcheck disable=SC2086
      SPMV_HIP_LIBRARY=$R/probes_build/libspmv_hip.so timeout -k 10 600 python3 -u ${step#probe:} \
          > "$O/$tag.log" 2> "$O/$tag.err" ;;
    exe:*)
      # shellcheck disable=SC2086
      timeout -k 10 600 ${step#exe:} > "$O/$tag.log" 2> "$O/$tag.err" ;;
    *)
      echo "unknown step $step" >&2; exit 64 ;;
  esac
  rc=$?
  echo "[$(date +%T)] step $tag rc=$rc" >&2
  if [ $rc -ne 0 ]; then
    exit $rc
  fi
done
