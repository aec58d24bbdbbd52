set -e
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD="python tools/bench_kernels.py --rounds 1 --reps 3 --variants wgrad_tap64=1 --layers L0\ 64->64,L2,L1\ 128->128"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pmc -o kt -- python tools/bench_kernels.py --rounds 1 --reps 3 --variants "wgrad_tap64=1" --layers "L0 64->64,L2,L1 128->128" > gpurun_out/pmc/kt.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -f csv -d gpurun_out/pmc -o sq -- python tools/bench_kernels.py --rounds 1 --reps 3 --variants "wgrad_tap64=1" --layers "L0 64->64,L2,L1 128->128" > gpurun_out/pmc/sq.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmc -o fetch -- python tools/bench_kernels.py --rounds 1 --reps 3 --variants "wgrad_tap64=1" --layers "L0 64->64,L2,L1 128->128" > gpurun_out/pmc/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmc -o write -- python tools/bench_kernels.py --rounds 1 --reps 3 --variants "wgrad_tap64=1" --layers "L0 64->64,L2,L1 128->128" > gpurun_out/pmc/write.log 2>&1
ls gpurun_out/pmc
