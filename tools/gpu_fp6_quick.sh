set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-5 91 92}; do timeout -k 10 60 python3 tools/gemm_one.py fp6 $v 65536 8192 8192 5 || exit 1; done
