# PMC passes (one counter group per run) over one GEMM: bash tools/gpu_pmc_gemm.sh KIND VARIANT M N K TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
KIND=$1; V=$2; M=$3; N=$4; K=$5; TAG=$6
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_$TAG
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_$TAG/$name -o $name --output-format csv -- python3 $R/tools/gemm_one.py $KIND $V $M $N $K 3 > $R/gpurun_out/pmc_$TAG/$name.log 2>&1 || { echo "PMC $name FAIL"; tail -5 $R/gpurun_out/pmc_$TAG/$name.log; return 1; }
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS && \
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run sq2 SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE && \
echo "PMC $TAG done"
