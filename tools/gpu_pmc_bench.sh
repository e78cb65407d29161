# PMC passes (one counter group per run) over one step of a bench config:
#   bash tools/gpu_pmc_bench.sh TAG KERNEL_SUBSTRING [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; SUB=$2; shift 2
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcb_$TAG
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmcb_$TAG/$name -o $name --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-kernel-timing $BENCH_ARGS > $R/gpurun_out/pmcb_$TAG/$name.log 2>&1 || { echo "PMC $name FAIL"; tail -5 $R/gpurun_out/pmcb_$TAG/$name.log; return 1; }
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM && \
run sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
python3 $R/tools/pmc_table.py $R/gpurun_out/pmcb_$TAG "$SUB"
