#!/bin/bash
# SQ counters of k_snappy on a short C3 bench run (one --pmc pass)
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --config c3 --steps 1 --warmup 0 --no-cpu --no-pmc > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc_sn -o run -- python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu --no-pmc > gpurun_out/pmc_sn.log 2>&1
