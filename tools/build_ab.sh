# Build libbnn.so from the csrc/ of a git revision into ab/<tag>/libbnn.so (A/B kernel timing on the
# box: BNN_LIB=ab/<tag>/libbnn.so python bench.py ...).  ab/ is git-ignored.
#   bash tools/build_ab.sh TAG REV
set -e
TAG=$1; REV=$2
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/ab/src_$TAG
rm -rf "$D"; mkdir -p "$D"
for f in $(git -C "$R" ls-tree --name-only "$REV" distributed-mnist-bnns_amd/csrc/); do
  git -C "$R" show "$REV:$f" > "$D/$(basename "$f")"
done
make -C "$D" -j8 OUT="$R/ab/$TAG/libbnn.so" OBJDIR="$R/ab/obj_$TAG" > "$R/ab/build_$TAG.log" 2>&1
echo "built $R/ab/$TAG/libbnn.so from $REV"
