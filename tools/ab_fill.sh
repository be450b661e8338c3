set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 64 128 256 512; do
IMPLISOLID_FILL_BLOCK=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab$m -o run -- python bench.py --steps 20 --skip-256 --skip-config5 --skip-ob02 --no-cpu-baseline > gpurun_out/ab$m.json 2>gpurun_out/ab$m.err
done
