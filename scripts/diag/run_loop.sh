# configs[4]: the 30k-iteration training loop through the C++ loop executable at 1080p
set -o pipefail
timeout -k 10 1000 python -u bench.py --mode loop --loop-engine cpp --loop-size 1920x1080 --loop-views 64 \
  --loop-gt ${LOOP_GT:-12000000} --loop-init ${LOOP_INIT:-400000} --loop-texture ${LOOP_TEX:-1.0} \
  --iters ${LOOP_ITERS:-30000} > gpurun_out/r03_bench_loop.json 2> gpurun_out/r03_bench_loop.err
rc=$?; tail -3 gpurun_out/r03_bench_loop.err; cat gpurun_out/r03_bench_loop.json; exit $rc
