#!/bin/bash
# round 6: the LDS word reader's pairs as one ds_read_b64 at 4-byte-aligned
# addresses (A/B build) against ds_read2_b32: C2 and C3 modes that read key
# bytes from LDS, library A B x 2, every output against host samples
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_ab_libs.sh ${1:-r06w} C2,C3 fnv1a_64,murmur,hsieh,one_at_a_time 0 twemproxy_amd/libnc_gpuhash.so abl/libnc_ldsb64.so 2
