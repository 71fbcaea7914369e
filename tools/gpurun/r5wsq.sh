#!/bin/bash
# Wave encoder: SQ counters for a lone wave (1 x 64 KiB) and a loaded chip
# (4096 x 64 KiB, every message on the wave encoder).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5wsq
rm -rf $O; mkdir -p $O
for n in 1 4096; do
  FSG_NOSTAMPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq_$n -o sq -- python3 tools/wstamps.py $n 65536 > $O/sq_$n.log 2>&1 || { tail -20 $O/sq_$n.log; exit 1; }
  echo "== n=$n"; grep messages $O/sq_$n.log
  python3 tools/pmc_sq.py $(find $O/sq_$n -name "*counter_collection.csv" | head -1) | grep -A12 encode_wave
  FSG_NOSTAMPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG --output-format csv -d $O/sq2_$n -o sq -- python3 tools/wstamps.py $n 65536 > $O/sq2_$n.log 2>&1 || { tail -20 $O/sq2_$n.log; exit 1; }
  python3 tools/pmc_sq.py $(find $O/sq2_$n -name "*counter_collection.csv" | head -1) | grep -A12 encode_wave
done
