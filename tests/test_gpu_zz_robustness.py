"""GPU robustness cases that run after the parity suites: caller errors the
library must survive without hanging or faulting (results unspecified)."""
import numpy as np
import pytest

import twemproxy_amd as t

from .test_gpu_dispatch import to_dev

pytestmark = pytest.mark.gpu


# (points, variant bits): 1000 points take the packed LDS continuum on the
# grouped pipeline; 1000 with bit 27 and 3000 take the 5-byte LDS form; the
# grouped pipeline with bit 25 searches the L2 continuum behind its LDS bucket
# index; bit 29 the workgroup pipeline, bit 28 the wave ring (LDS continuum
# with a 257-entry index); 6000 points exceed every LDS budget (hash launch,
# then the dispatch kernel's bucket search)
UNSORTED_CASES = [(1000, 0), (1000, (1 << 30) | (1 << 27)), (3000, 0), (3000, (1 << 30) | (1 << 25)),
                  (3000, 1 << 29), (3000, 1 << 28), (6000, 0)]


@pytest.mark.parametrize("npoints,var", UNSORTED_CASES, ids=[f"{n}-{v:#x}" for n, v in UNSORTED_CASES])
def test_ketama_unsorted_continuum_terminates(gpu, npoints, var):
    """A continuum that is not sorted is a caller error (ketama_update sorts,
    src/hashkit/nc_ketama.c:198), but every ketama search must still end
    inside the continuum: bucket spans are clamped to n (bucket_span), and
    the packed search also stops at its eight sentinels. The results are
    unspecified; the launch must return server indices."""
    import torch

    from twemproxy_amd import _lib as L

    spec = t.CONFIGS["C2"]["spec"]
    n = 1 << 17
    keys, off = t.synth_host(spec, 5, n)
    kd, od = to_dev(keys, off)
    rng = np.random.default_rng(17)
    vals = rng.integers(0, 1 << 32, size=npoints, dtype=np.uint64).astype(np.uint32)  # not sorted
    idx = rng.integers(0, 8, size=vals.size).astype(np.uint32)
    cd = t.continuum_device(idx, vals)
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        got = t.server_idx_device("fnv1a_64", "ketama", kd, od, cd, 8, shape=spec.shape(int(off[-1])))
        torch.cuda.synchronize()
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)
    assert int(got.cpu().numpy().view(np.uint32).max()) < 8
