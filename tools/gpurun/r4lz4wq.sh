#!/bin/bash
# SQ counters of the LZ4 decode kernels on one 2 MiB body (wave walk).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4wq
rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/a -o a -- python3 tools/lz4_bench.py --n 1 --size 2097152 --steps 1 --no-cpu --no-pipelined --two-pass-only > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
python3 tools/pmc_sq.py $(find $O/a -name "*counter_collection.csv" | head -1) | grep -A12 "lz4_index\|lz4_exec"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG SQ_INST_CYCLES_SALU --output-format csv -d $O/b -o b -- python3 tools/lz4_bench.py --n 1 --size 2097152 --steps 1 --no-cpu --no-pipelined --two-pass-only > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python3 tools/pmc_sq.py $(find $O/b -name "*counter_collection.csv" | head -1) | grep -A10 "lz4_index_big"
