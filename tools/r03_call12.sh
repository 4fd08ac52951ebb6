#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c12
mkdir -p $O
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; df -h /tmp /dev/shm; mount | grep -E " /tmp | /dev/shm ") > $O/env.log 2>&1 || true
timeout -k 10 300 python tools/host_read_probe.py --frames 1024 > $O/hrp_tmp.log 2>&1
timeout -k 10 300 python tools/host_read_probe.py --frames 1024 --dir /dev/shm > $O/hrp_shm.log 2>&1
