# FETCH_SIZE / WRITE_SIZE passes (one counter per run) over one BinCNN bench step, summarised into
# gpurun_out/$TAG_pmc_traffic.json for bench.py's roofline.traffic.  bash tools/gpu_pmc_cnn.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmcc_$TAG && mkdir -p $R/gpurun_out/pmcc_$TAG
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $R/gpurun_out/pmcc_$TAG/$c -o cnn --output-format csv -- python3 $R/bench.py --config cnn --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/pmcc_$TAG/$c.log 2>&1 || { echo "PMC $c FAIL"; tail -5 $R/gpurun_out/pmcc_$TAG/$c.log; exit 1; }
done
python3 $R/tools/pmc_summary.py --fetch $R/gpurun_out/pmcc_$TAG/FETCH_SIZE --write $R/gpurun_out/pmcc_$TAG/WRITE_SIZE --out $R/gpurun_out/${TAG}_pmc_traffic.json && echo PMC OK
