#!/bin/bash
# round 4, GPU call 18: the 6000-record deep-list case against the oracle with and without chunk
# merging (rel-L2 of image and gradients) -- merge effect vs f32 drift over deep faint lists
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_18
mkdir -p $O
cd $R
for v in base nomerge old; do
  for c in "2000 0.005" "6000 0.0045" "6000 0.02"; do
    if [ $v = base ]; then
      timeout -k 10 120 python -u tests/diag_deep_lists.py $c >> $O/rel.txt 2>> $O/rel.err || exit $?
    else
      GSR_HIP_LIB=$R/3d_gaussian_splatting_amd/lib/variants/$v/libgsr_hip.so timeout -k 10 120 python -u tests/diag_deep_lists.py $c >> $O/rel.txt 2>> $O/rel.err || exit $?
    fi
  done
done
