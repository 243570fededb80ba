# Build the library of a git revision (default HEAD) as sctools_amd/libsctools_hip_base.so, for
# same-box A/B runs against the working tree's library (SCTOOLS_HIP_LIB selects it).
#   bash tools/build_base_lib.sh [rev]
set -eu
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" sctools_amd/csrc include | tar -x -C "$T"
make -s -j8 -C "$T/sctools_amd/csrc" ../libsctools_hip.so
cp "$T/sctools_amd/libsctools_hip.so" "$ROOT/sctools_amd/libsctools_hip_base.so"
rm -rf "$T"
echo "built sctools_amd/libsctools_hip_base.so from $REV"
