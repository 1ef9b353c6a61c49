#!/bin/bash
# Where this process may run and allocate, and where the GPU sits (NUMA A/B context).
grep -E "Cpus_allowed_list|Mems_allowed_list" /proc/self/status
for n in /sys/devices/system/node/node*; do echo "$(basename $n) cpus $(cat $n/cpulist)"; done
python3 -c "import ctypes; L=ctypes.CDLL('rclone_amd/librclone_crypt.so'); print('device0_numa_node', L.xs_device_numa_node(0))"
nproc
