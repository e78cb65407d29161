# cost of device-scope compact-input loads in the BatchNorm2d kernels (A/B on the BinCNN step);
# the MLP paths (config 2, small MLP) under 4-process contention with the default build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
for v in default coh; do
  if [ $v = coh ]; then export BNN_LIB=$R/abv/coh/libbnn.so; else unset BNN_LIB; fi
  timeout -k 10 200 python -u bench.py --config cnn --steps 50 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_r_cnn_$v.log 2>&1; rc=$?
  echo "== $v cnn bench exit $rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05_r_cnn_$v.log; ok $rc
done
unset BNN_LIB
timeout -k 10 400 python -u tools/race_probe.py 4 30 config2 mlp > gpurun_out/r05_r_race_mlp.log 2>&1; rc=$?
echo "== MLP race exit $rc"; grep -v amdgpu gpurun_out/r05_r_race_mlp.log | cut -c1-200 | tail -20; ok $rc
