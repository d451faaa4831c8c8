# Build a variant of the library with extra flags for ONE source file (the
# rest from build/): bash tools/build_variant.sh <name> <source-stem> "<flags>"
# -> binquant_amd/lib/variants/lib_<name>.so  (A/B runs: BQ_LIB_PATH=...)
set -e
cd "$(dirname "$0")/.."
NAME=$1; STEM=$2; FLAGS=$3
make -s -j8 >/dev/null
mkdir -p build/variants binquant_amd/lib/variants
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -std=c++17 -Iinclude -Ibinquant_amd/csrc -Wall -Wno-unused-function $FLAGS -c binquant_amd/csrc/$STEM.hip -o build/variants/${STEM}_$NAME.o
OBJS=$(ls build/*.o | grep -v "/$STEM.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o binquant_amd/lib/variants/lib_$NAME.so $OBJS build/variants/${STEM}_$NAME.o -lhiprtc
echo binquant_amd/lib/variants/lib_$NAME.so
