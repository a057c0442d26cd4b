"""The device-generated DB spec (pm_batchpir_create_synth, include/pacmann.h):
pacmann_amd.synth_rows against a pure-Python restatement of splitmix64."""
import numpy as np

M64 = (1 << 64) - 1


def sm64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def test_synth_rows_spec():
    from pacmann_amd import synth_rows
    seed, E = 41, 80
    ids = [0, 1, 12_345_678, 10**9 - 1]
    got = synth_rows(seed, ids, E)
    k = sm64(seed + 9)
    for i, r in enumerate(ids):
        want = [sm64(k ^ (r * E + w)) for w in range(E)]
        assert got[i].tolist() == want
    assert got.dtype == np.uint64 and got.shape == (4, E)
