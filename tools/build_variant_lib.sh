# Build the working tree's library with extra -D flags as sctools_amd/libsctools_hip_<name>.so
# (timing-only variants for same-box A/B runs; SCTOOLS_HIP_LIB selects one).
#   bash tools/build_variant_lib.sh NAME "-DFLAG ..."
set -eu
NAME=$1
FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cp -r "$ROOT/sctools_amd/csrc" "$ROOT/include" "$T/" 2>/dev/null || true
mkdir -p "$T/sctools_amd" && mv "$T/csrc" "$T/sctools_amd/csrc" && rm -rf "$T/sctools_amd/csrc/build"
make -s -j8 -C "$T/sctools_amd/csrc" ../libsctools_hip.so FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $FLAGS"
cp "$T/sctools_amd/libsctools_hip.so" "$ROOT/sctools_amd/libsctools_hip_$NAME.so"
rm -rf "$T"
echo "built sctools_amd/libsctools_hip_$NAME.so"
