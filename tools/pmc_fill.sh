set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --steps 5 --warmup 1 --skip-256 --skip-config5 --skip-ob02 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pf_sq -o run -- $B > /dev/null 2>gpurun_out/pf_sq.err
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum --output-format csv -d gpurun_out/pf_tcc -o run -- $B > /dev/null 2>gpurun_out/pf_tcc.err
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pf_ta -o run -- $B > /dev/null 2>gpurun_out/pf_ta.err
