#!/bin/bash
# Compile-time-matrix encode (kernels_xb.hip): the parity suite, then its A/B (W = 1 / 2 dwords
# per lane, SEC_XB=0 = the v_perm kernel) on the wide policy shapes at 1 MiB and 16 MiB chunks.
set -o pipefail
bash tools/gpu_tests.sh tests/test_gpu_parity.py && VARIANTS=base,base@SEC_XB_W=2,base@SEC_XB=0 WORKLOADS="1024,1048576,32,48 256,1048576,64,96 16,16777216,64,96 64,16777216,32,48" bash tools/gpu_ab.sh
