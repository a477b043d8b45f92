set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for p in 0 1; do
TAG="prio=$p rep=$rep" BV_COPY_PRIO=$p timeout -k 10 200 python -u tools/host_entry_stalls.py 2>/dev/null | grep median
done; done
