"""GPU robustness cases that run after the parity suites: caller errors the
library must survive without hanging or faulting (results unspecified)."""
import numpy as np
import pytest

import twemproxy_amd as t

from .test_gpu_dispatch import to_dev

pytestmark = pytest.mark.gpu


def test_ketama_unsorted_continuum_terminates(gpu):
    """A continuum that is not sorted is a caller error (ketama_update sorts,
    src/hashkit/nc_ketama.c:198), but the packed LDS search must still end:
    its bucket starts are clamped to n and four sentinels stop the scan. The
    results are unspecified; the launch must return server indices."""
    import torch

    spec = t.CONFIGS["C2"]["spec"]
    n = 1 << 17
    keys, off = t.synth_host(spec, 5, n)
    kd, od = to_dev(keys, off)
    rng = np.random.default_rng(17)
    vals = rng.integers(0, 1 << 32, size=1000, dtype=np.uint64).astype(np.uint32)  # not sorted
    idx = rng.integers(0, 8, size=vals.size).astype(np.uint32)
    cd = t.continuum_device(idx, vals)
    got = t.server_idx_device("fnv1a_64", "ketama", kd, od, cd, 8, shape=spec.shape(int(off[-1])))
    torch.cuda.synchronize()
    assert int(got.cpu().numpy().view(np.uint32).max()) < 8
