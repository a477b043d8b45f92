# Build libbabbleverify.so with extra -D flags into $1 (A/B experiments on
# one GPU box): tools/build_variant.sh gpurun_var/x.so -DFOO=0
set -e
out=$1; shift
d=$(mktemp -d)
cd "$(dirname "$0")/../babble_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable $*"
/opt/rocm/bin/hipcc $F -c kernels.hip -o $d/k.o &
for f in bv_api bv_group bv_events hostparse; do /opt/rocm/bin/hipcc $F -x hip -c $f.cpp -o $d/$f.o & done
wait
cd - > /dev/null
mkdir -p "$(dirname "$out")"
/opt/rocm/bin/hipcc $F -shared -o "$out" $d/*.o -ldl -lpthread
rm -rf $d
