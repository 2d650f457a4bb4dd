set -o pipefail
mkdir -p gpurun_out/cprof && cd gpurun_out/cprof && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > counters.txt 2>&1 || true
cd ../..
A="24 64 64 3 1 1 48 160 1 1 20"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof/t -o run -- python tools/conv_prof.py $A > gpurun_out/cprof/t.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/cprof/p1 -o run -- python tools/conv_prof.py $A > gpurun_out/cprof/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/cprof/p2 -o run -- python tools/conv_prof.py $A > gpurun_out/cprof/p2.log 2>&1
