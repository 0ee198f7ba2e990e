# Build sweep-kernel variant libraries (experiments only) into kwok_amd/lib/variants/.
#   bash tools/build_variants.sh lut:-DKWOK_MATCH_LUT=1 ldst:-DKWOK_LDS_TABLE=1,-DKWOK_MATCH_LUT=1
# Each argument is name:comma-separated hipcc defines.
set -e
cd "$(dirname "$0")/.."
mkdir -p kwok_amd/lib/variants
rm -f kwok_amd/lib/variants/*.so
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value -I include \
    ${defs//,/ } -o kwok_amd/lib/variants/libkwok_$name.so kwok_amd/csrc/engine.hip &
done
wait
ls kwok_amd/lib/variants
