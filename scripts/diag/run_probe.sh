set -o pipefail
probe() {  # name gt init tex scale
  timeout -k 10 200 python -u bench.py --mode loop --loop-engine cpp --loop-size 1920x1080 --loop-views 32 \
    --loop-gt $2 --loop-init $3 --loop-texture $4 --loop-gt-scale $5 --iters 3100 > gpurun_out/r03_probe_$1.json 2> gpurun_out/r03_probe_$1.err || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['final_gaussians'], d['gaussians_after_densify'][-3:], d['loss_curve'][-1])" gpurun_out/r03_probe_$1.json
}
probe A 12000000 400000 1.0 0.012 && probe B 12000000 400000 1.0 0.005 && probe C 12000000 200000 2.0 0.005 && probe D 20000000 300000 1.5 0.004
