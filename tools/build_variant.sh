# Build libbabbleverify.so with extra -D flags into $1 (A/B experiments on
# one GPU box): tools/build_variant.sh gpurun_var/x.so -DFOO=0
# The sources are copied to a scratch directory and built by their own
# Makefile (host-only files with the host compiler), the extra flags added to
# the device compile.  With BV_REV=<git revision> that revision is built.
set -e
out=$(realpath -m "$1"); shift
root="$(cd "$(dirname "$0")/.." && pwd)"
d=$(mktemp -d)
if [ -n "$BV_REV" ]; then
  git -C "$root" archive "$BV_REV" babble_amd/csrc include | tar -x -C $d
else
  mkdir -p $d/babble_amd && cp -r "$root/babble_amd/csrc" $d/babble_amd/ && cp -r "$root/include" $d/
  rm -rf $d/babble_amd/csrc/obj
fi
mkdir -p "$(dirname "$out")"
make -s -C $d/babble_amd/csrc -j8 OUT="$out" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable $*"
rm -rf $d
