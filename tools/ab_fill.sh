set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab -o run -- python bench.py --steps 20 --skip-256 --skip-config5 --skip-ob02 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err
timeout -k 10 300 python bench.py --steps 50 --skip-256 --skip-config5 --skip-ob02 --no-cpu-baseline > gpurun_out/ab2.json 2>gpurun_out/ab2.err
