# Round-3: PMC passes (SQ busy/wait/instruction mix, LDS) over the wide step's quantising BN backward.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
SUB=bn_bwd_apply_q6
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcq
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmcq/$name -o $name --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/pmcq/$name.log 2>&1 || { echo "PMC $name FAIL"; tail -5 $R/gpurun_out/pmcq/$name.log; return 1; }
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM && \
run sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
run sq3 SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_INSTS_MFMA SQ_WAVES && \
python3 $R/tools/pmc_table.py $R/gpurun_out/pmcq "$SUB"
