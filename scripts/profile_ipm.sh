#!/bin/bash
# Per-sweep profile of an IPM workload (diagnostic library built with -DSRBD_IPM_SPLIT=1:
# RB, F1, B2, F2 as separate launches): kernel trace, FETCH_SIZE, WRITE_SIZE and two SQ
# passes, each its own rocprofv3 run.  Usage: profile_ipm.sh TAG WORKLOAD LIB
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=$1; W=$2; LIB=$3
OUT=gpurun_out/prof_${TAG}_${W}
mkdir -p $OUT
export SRBD_QP_LIB=$LIB
BA="--workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline --no-host-path --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BA > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $BA > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $BA > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq1 -o run -- python3 bench.py $BA > $OUT/sq1.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $BA > $OUT/sq2.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/tcc -o run -- python3 bench.py $BA > $OUT/tcc.log 2>&1 || exit $?
find $OUT -name "*.csv" | wc -l
