set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/r02/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r02/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/r02/bench_c2.json 2> gpurun_out/r02/bench_c2.err || exit 1
for k in 2 4 8; do timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --sim-world $k --formats css,ell > gpurun_out/r02/bench_sim$k.json 2> gpurun_out/r02/bench_sim$k.err || exit 1; done
timeout -k 10 500 python bench.py --config c3 --steps 30 --warmup 5 --formats auto,csr,ell,ss,hyb,css > gpurun_out/r02/bench_c3.json 2> gpurun_out/r02/bench_c3.err || exit 1
timeout -k 10 600 python bench.py --config c4 --steps 20 --warmup 5 --formats auto,csr,dia > gpurun_out/r02/bench_c4.json 2> gpurun_out/r02/bench_c4.err || exit 1
echo all-done
