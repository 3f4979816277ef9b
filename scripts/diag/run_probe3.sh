set -o pipefail
probe() {  # name gt init tex scale iters
  timeout -k 10 300 python -u bench.py --mode loop --loop-engine cpp --loop-size 1920x1080 --loop-views 32 \
    --loop-gt $2 --loop-init $3 --loop-texture $4 --loop-gt-scale $5 --iters $6 > gpurun_out/r03_probe_$1.json 2> gpurun_out/r03_probe_$1.err || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['final_gaussians'], d['gaussians_after_densify'][-4:], d['loss_curve'][-1])" gpurun_out/r03_probe_$1.json
}
probe H 20000000 3000000 1.0 0.005 6100 && probe I 20000000 2000000 1.0 0.004 6100
