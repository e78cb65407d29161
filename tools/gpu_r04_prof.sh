# Round 4: rocprofv3 kernel-trace stats of the default bench step, then SQ PMC passes (instruction
# mix, busy / wait cycles) over every libbnn kernel of one step.  TAG names the output dirs;
# BENCH_ARGS (e.g. "--config cnn") picks another bench configuration.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04}
cd $R && mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o wide --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing $BENCH_ARGS > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-200
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1) 7 24 > $R/gpurun_out/prof_${TAG}_summary.txt || exit 1
head -26 $R/gpurun_out/prof_${TAG}_summary.txt | cut -c1-150
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_$TAG/$name -o $name --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-kernel-timing $BENCH_ARGS > $R/gpurun_out/pmc_$TAG/$name.log 2>&1 || { echo "PMC $name FAIL"; tail -5 $R/gpurun_out/pmc_$TAG/$name.log; return 1; }
}
[ "${PMC:-1}" = "1" ] || exit 0
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE && \
run sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA GRBM_GUI_ACTIVE && \
python3 $R/tools/pmc_table.py $R/gpurun_out/pmc_$TAG "bn_" > $R/gpurun_out/pmc_${TAG}_bn.txt && \
python3 $R/tools/pmc_table.py $R/gpurun_out/pmc_$TAG "" > $R/gpurun_out/pmc_${TAG}_all.txt && echo PMC OK
