# Build an A/B variant of libmplc_hip.so into gpurun_ab/<name>.so: bash scripts/build_variant.sh <name> [-DFLAG ...]
# (mnist_cnn.hip - or $VARIANT_SRC, a modified copy of csrc/$VARIANT_BASE.hip - recompiled with the extra flags,
# linked with the in-tree objects of the other sources)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
P=distributed-learning-contributivity_amd
mkdir -p gpurun_ab
python $P/build_native.py
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I $P/csrc ${VARIANT_FLAGS--fno-slp-vectorize} "$@" \
  -c ${VARIANT_SRC:-$P/csrc/mnist_cnn.hip} -o /tmp/variant_$NAME.o
objs=$(ls $P/build/*.o | grep -v "/${VARIANT_BASE:-mnist_cnn}.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o gpurun_ab/$NAME.so $objs /tmp/variant_$NAME.o
echo built gpurun_ab/$NAME.so
