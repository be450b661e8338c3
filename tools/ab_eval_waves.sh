# A/B of the eval kernel's occupancy request: default vs IMPLISOLID_EVAL_WAVES=8 (rocprof + bench each)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --steps 50 --skip-256 --skip-config5 --skip-ob02 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abw0 -o run -- $B > gpurun_out/abw0.json 2>gpurun_out/abw0.err
IMPLISOLID_EVAL_WAVES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abw8 -o run -- $B > gpurun_out/abw8.json 2>gpurun_out/abw8.err
timeout -k 10 300 $B > gpurun_out/abw0b.json 2>>gpurun_out/abw0.err
IMPLISOLID_EVAL_WAVES=8 timeout -k 10 300 $B > gpurun_out/abw8b.json 2>>gpurun_out/abw8.err
python tools/kstats.py gpurun_out/abw0 > gpurun_out/ksw0.txt
python tools/kstats.py gpurun_out/abw8 > gpurun_out/ksw8.txt
