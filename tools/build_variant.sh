# Build libbabbleverify.so with extra -D flags into $1 (A/B experiments on
# one GPU box): tools/build_variant.sh gpurun_var/x.so -DFOO=0
# With BV_REV=<git revision> the sources of that revision are built instead.
set -e
out=$(realpath -m "$1"); shift
d=$(mktemp -d)
src="$(dirname "$0")/../babble_amd/csrc"
if [ -n "$BV_REV" ]; then
  git -C "$(dirname "$0")/.." archive "$BV_REV" babble_amd/csrc include | tar -x -C $d
  src=$d/babble_amd/csrc
fi
cd "$src"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable $*"
/opt/rocm/bin/hipcc $F -c kernels.hip -o $d/k.o &
for f in *.cpp; do /opt/rocm/bin/hipcc $F -x hip -c $f -o $d/${f%.cpp}.o & done
wait
cd - > /dev/null
mkdir -p "$(dirname "$out")"
/opt/rocm/bin/hipcc $F -shared -o "$out" $d/*.o -ldl -lpthread
rm -rf $d
