# Like build_variant.sh but from an arbitrary (e.g. patched, uncommitted)
# copy of one source: bash tools/build_variant_src.sh <name> <stem> <path.hip> "<flags>"
set -e
cd "$(dirname "$0")/.."
NAME=$1; STEM=$2; SRC=$3; FLAGS=$4
make -s -j8 >/dev/null
mkdir -p build/variants binquant_amd/lib/variants
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -std=c++17 -Iinclude -Ibinquant_amd/csrc -Wno-unused-function $FLAGS -x hip -c $SRC -o build/variants/${STEM}_$NAME.o
OBJS=$(ls build/*.o | grep -v "/$STEM.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o binquant_amd/lib/variants/lib_$NAME.so $OBJS build/variants/${STEM}_$NAME.o -lhiprtc
echo binquant_amd/lib/variants/lib_$NAME.so
