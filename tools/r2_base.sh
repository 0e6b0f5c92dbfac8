set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2_base
cd $R
timeout -k 10 300 python3 -u bench.py --steps 50 --warmup 10 > gpurun_out/r2_base/bench.json 2> gpurun_out/r2_base/bench.err || exit $?
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_base/trace -o run -- python3 $R/bench.py --no-cpu --formats auto --steps 50 --warmup 10 > $R/gpurun_out/r2_base/bench_trace.json 2> $R/gpurun_out/r2_base/trace.err
