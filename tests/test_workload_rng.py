"""The synthetic-workload generator's specification (oracle/philox.py), on CPU.

Philox-4x32-10 is pinned to the published known-answer vectors of its
authors (Random123 kat_vectors); the derived hand inputs must be keyed by the
global hand index (a shard reproduces the global batch) and have the stated
distributions.  tests/test_gpu_workloads.py checks the device generator
against this restatement."""
import numpy as np

from oracle import philox


def test_philox_known_answers():
    kat = [([0, 0, 0, 0], (0, 0), [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
           ([0xffffffff] * 4, (0xffffffff, 0xffffffff), [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
           ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], (0xa4093822, 0x299f31d0),
            [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1])]
    for ctr, key, want in kat:
        got = philox.philox4x32_10(np.array(ctr, dtype=np.uint32), *key)
        assert [int(x) for x in got] == want


def test_shard_invariance_and_distribution():
    full = philox.synthetic_inputs(1002, 0, 4000)
    part = philox.synthetic_inputs(1002, 1234, 500)
    for k in ("betas", "pose", "trans"):
        assert np.array_equal(full[k][1234:1734], part[k])
    assert abs(full["betas"].mean()) < 0.05 and abs(full["betas"].std() - 1.0) < 0.03
    assert abs(full["pose"].mean()) < 0.02 and abs(full["pose"].std() - 0.5) < 0.02
    assert full["trans"].min() > -1 and full["trans"].max() < 1
    assert abs(full["trans"].mean()) < 0.05
    other = philox.synthetic_inputs(1003, 0, 10)
    assert not np.array_equal(other["betas"], full["betas"][:10])


def test_high_index_words_use_the_upper_counter():
    a = philox.words(7, 2 ** 32 + 5, 1)
    b = philox.words(7, 5, 1)
    assert not np.array_equal(a, b)
