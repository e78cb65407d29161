# Round 4 A/B: kernel-trace stats of the default bench step for the libraries named in LIBS
# (TAG=path pairs), each run twice in alternation.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for round in 1 2; do
  for spec in $LIBS; do
    tag=${spec%%=*}; lib=${spec#*=}
    BNN_LIB=$R/$lib bash tools/gpu_stats.sh ab_${tag}_$round > gpurun_out/ab_${tag}_$round.txt 2>&1 || { echo "AB $tag FAIL"; tail -5 gpurun_out/ab_${tag}_$round.txt; exit 1; }
    echo "== $tag round $round: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_ab_${tag}_$round.log)"
    grep -E "bn_head|q6_k<10|${AB_GREP:-bn_head}" gpurun_out/ab_${tag}_$round.txt | cut -c1-120
  done
done
