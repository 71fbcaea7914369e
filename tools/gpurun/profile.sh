#!/bin/bash
# Profile recipe run on the GPU box (gpurun): bench lines for every workload,
# rocprofv3 kernel trace/stats and the PMC traffic passes (FETCH_SIZE and
# WRITE_SIZE in separate runs) for the default workload and the C2
# calibration case.  Each GPU step is time-limited; the chain stops at the
# first failure.  Results land in gpurun_out/prof/.
set -e
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
B="python bench.py"
timeout -k 10 300 $B > $O/bench_c3d.json 2> $O/bench_c3d.err
timeout -k 10 300 $B --workload c2-decompress --steps 20 --warmup 3 > $O/bench_c2d.json 2> $O/bench_c2d.err
timeout -k 10 300 $B --workload cm-decompress --steps 5 --warmup 1 > $O/bench_cmd.json 2> $O/bench_cmd.err
timeout -k 10 300 $B --workload c3-compress --steps 3 --warmup 1 > $O/bench_c3c.json 2> $O/bench_c3c.err
timeout -k 10 300 $B --workload c5-compress --steps 3 --warmup 1 > $O/bench_c5c.json 2> $O/bench_c5c.err
cd $O
Q="--steps 3 --warmup 1 --no-e2e --no-cpu-baseline --verify-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d kt -o kt -- python ../../bench.py $Q > kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ktm -o ktm -- python ../../bench.py --workload cm-decompress $Q > ktm.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d f3 -o f3 -- python ../../bench.py $Q > f3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d w3 -o w3 -- python ../../bench.py $Q > w3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d f2 -o f2 -- python ../../bench.py --workload c2-decompress $Q > f2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d w2 -o w2 -- python ../../bench.py --workload c2-decompress $Q > w2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS --output-format csv -d sq -o sq -- python ../../bench.py $Q > sq.log 2>&1
echo done
