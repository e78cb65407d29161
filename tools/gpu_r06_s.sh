# Round 6, call S: conv1's fused filter gradient (conv_bwd_filter_c1bn_k) with the pooled-row LDS pitch
# (bnn_conv_set_c1bn_pitch 1, default) vs the old pitch (0): BinCNN tests, interleaved graph-step
# timings in one build, kernel stats of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_cnn_parity.py \
  tests/test_gpu_parity.py tests/test_gpu_conv_popc.py tests/test_gpu_parallel.py \
  > gpurun_out/r06_s_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_s_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_s_gpu_tests.log | tail -1
run() {   # pitch tag args...
  local p=$1 tag=$2; shift 2
  timeout -k 10 300 python -c "
import sys, runpy
sys.path.insert(0, 'distributed-mnist-bnns_amd')
from bnn_amd import _lib as L
L.call('bnn_conv_set_c1bn_pitch', $p)
sys.argv = ['bench.py'] + sys.argv[1:]
runpy.run_path('bench.py', run_name='__main__')" "$@" > gpurun_out/r06_s_$tag.log 2>&1 || { echo RUN $tag FAIL; tail -5 gpurun_out/r06_s_$tag.log; return 1; }
}
for rep in 1 2; do
  for p in 0 1; do
    run $p g_p${p}_$rep --config cnn --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin || exit 1
    echo "graph pitch $p rep $rep: $(tail -1 gpurun_out/r06_s_g_p${p}_$rep.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
cd /tmp && export TMPDIR=/tmp
for p in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06s_p$p -o cnng --output-format csv -- python3 -c "
import sys, runpy
sys.path.insert(0, '$R/distributed-mnist-bnns_amd')
from bnn_amd import _lib as L
L.call('bnn_conv_set_c1bn_pitch', $p)
sys.argv = ['bench.py', '--config', 'cnn', '--graph', '--steps', '100', '--warmup', '5', '--no-cpu-baseline', '--no-gpu-torch', '--no-dropin', '--no-kernel-timing']
runpy.run_path('$R/bench.py', run_name='__main__')" > $R/gpurun_out/r06_s_prof_p$p.log 2>&1 || { echo PROF FAIL; tail -5 $R/gpurun_out/r06_s_prof_p$p.log; exit 1; }
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06s_p$p -name 'cnng_kernel_stats.csv' | head -1) 105 40 > $R/gpurun_out/r06_s_cnng_stats_p$p.txt
  echo "pitch $p:"; grep -E "c1bn|kernel time" $R/gpurun_out/r06_s_cnng_stats_p$p.txt | cut -c1-130
done
