#!/bin/bash
# round 6: two A/B builds in one call — the short-key kernel's offsets with the
# default cache policy (C3), the grouped tile's bound dwords likewise (C2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_ab_libs.sh r06l C3 crc32,jenkins,one_at_a_time,murmur 0 twemproxy_amd/libnc_gpuhash.so abl/libnc_shortoff.so 2 || exit 1
bash tools/gpu_r6_gsbound.sh r06m || exit 1
