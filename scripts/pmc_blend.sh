#!/bin/bash
# Occupancy / issue counters for the blend kernels (one PMC group per pass).
cd /tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc2
mkdir -p $OUT
BENCH="python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage-events"
timeout -k 10 240 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 -d $OUT/a -o a --output-format csv -- $BENCH > $OUT/a.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES -d $OUT/b -o b --output-format csv -- $BENCH > $OUT/b.log 2>&1
echo pmc_rc=$?
