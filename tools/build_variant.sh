# Build libbnn.so from the working tree's csrc/ with extra compiler flags into ab/<tag>/libbnn.so
# (timing-only variants, e.g. -DQ6_DIAG_NOSTORE).  ab/ is git-ignored.
#   bash tools/build_variant.sh TAG "-DFLAG ..."
set -e
TAG=$1; EXTRA=$2
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/ab/src_$TAG
rm -rf "$D"; mkdir -p "$D"
cp $R/distributed-mnist-bnns_amd/csrc/* "$D/"
make -C "$D" -j8 OUT="$R/ab/$TAG/libbnn.so" OBJDIR="$R/ab/obj_$TAG" \
  CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fvisibility=hidden $EXTRA" > "$R/ab/build_$TAG.log" 2>&1
echo "built $R/ab/$TAG/libbnn.so ($EXTRA)"
