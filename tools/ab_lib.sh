#!/bin/bash
# Build the library of git revision REV (default HEAD) as ab/libensvs_<REV>.so beside the
# working-tree build, for A/B timing: ENSVS_LIB=ab/libensvs_<REV>.so python3 tools/...
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
D=$(mktemp -d)
git archive "$REV" ensemble_svs_with_interactions_amd/csrc include | tar -x -C "$D"
mkdir -p ab
for f in "$D"/ensemble_svs_with_interactions_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$D"/ensemble_svs_with_interactions_amd/csrc \
    -I"$D"/include -c "$f" -o "$D/$(basename "$f" .hip).o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "ab/libensvs_$REV.so" "$D"/*.o
rm -rf "$D"
echo "ab/libensvs_$REV.so"
