#!/bin/bash
# SQ instruction-mix / utilisation counters (two --pmc passes, each within the
# per-block limits of MI355X_MICROARCH.md) for one bench workload.
# Usage: profile_sq.sh TAG WORKLOAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=$1; W=$2
OUT=gpurun_out/prof_${TAG}_${W}
mkdir -p $OUT
BA="--workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-pipeline --no-host-path --no-secondary"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq1 -o run -- python3 bench.py $BA > $OUT/sq1.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F32 SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $BA > $OUT/sq2.log 2>&1 || exit $?
find $OUT -name "*counter_collection.csv"
