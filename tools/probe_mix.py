#!/usr/bin/env python3
"""Same-process HBM probes over a C2-sized buffer (2.2 GB): the 16-byte read
with the default and the non-temporal policy, and the read+write mix of a
hash kernel (nt reads plus one streaming 16-byte store per 128 bytes read,
nc_gpuhash_probe_mix). Three interleaved rounds; one JSON line per round."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import twemproxy_amd as t

    buf = torch.randint(0, 256, (2200 * 1000 * 1000 // 16 * 16,), dtype=torch.uint8, device="cuda")
    t.probe_read_gbs(buf, 3)
    t.probe_mix_gbs(buf, 3)
    for r in range(3):
        print(json.dumps({"round": r, "bytes": buf.numel(), "read_gbs": round(t.probe_read_gbs(buf, 20), 1),
                          "read_nt_gbs": round(t.probe_read_gbs(buf, 20, nt=True), 1),
                          "mix_gbs": round(t.probe_mix_gbs(buf, 20), 1),
                          "mix_ld_default_gbs": round(t.probe_mix_gbs(buf, 20, policy=1), 1),
                          "mix_st_default_gbs": round(t.probe_mix_gbs(buf, 20, policy=2), 1),
                          "mix_both_default_gbs": round(t.probe_mix_gbs(buf, 20, policy=3), 1)}), flush=True)


if __name__ == "__main__":
    main()
