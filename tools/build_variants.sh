# Build sweep-kernel variant libraries (experiments only) into kwok_amd/lib/variants/.
#   bash tools/build_variants.sh 8 16      # KWOK_GROUP values
set -e
cd "$(dirname "$0")/.."
mkdir -p kwok_amd/lib/variants
rm -f kwok_amd/lib/variants/*.so
for g in "$@"; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value -I include \
    -DKWOK_GROUP=$g -o kwok_amd/lib/variants/libkwok_g$g.so kwok_amd/csrc/engine.hip &
done
wait
ls kwok_amd/lib/variants
