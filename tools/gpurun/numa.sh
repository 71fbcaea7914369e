#!/bin/bash
# H2D/D2H by NUMA node of the allocating process (tools/h2d_numa_probe.py).
ls -d /sys/devices/system/node/node* | wc -l
for n in $(ls -d /sys/devices/system/node/node* | sed 's/.*node//'); do
  timeout -k 10 120 python tools/h2d_numa_probe.py $n || exit 1
done
for d in /sys/class/drm/card*/device/numa_node; do echo "$d $(cat $d)"; done 2>/dev/null | head -4
