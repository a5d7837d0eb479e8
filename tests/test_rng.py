"""The numpy restatement of the device dropout generator (tests/philox_ref.py)
against the Random123 Philox4x32-10 known-answer vectors, and the word ->
uniform mapping."""
import numpy as np

from philox_ref import dropout_uniform_ref, philox4x32_10


def test_philox_known_answers():
    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for c, k, want in kat:
        got = tuple(int(w) for w in philox4x32_10(*c, *k))
        assert got == want, [hex(x) for x in got]


def test_uniform_range_and_layout():
    u = dropout_uniform_ref(10001, seed=1234, step=7, salt=1)
    assert u.dtype == np.float32 and u.shape == (10001,)
    assert (u >= 0).all() and (u < 1).all()
    assert abs(float(u.mean()) - 0.5) < 0.01
    # element i is word i % 4 of counter block i // 4
    w = philox4x32_10(2, 0, 1, 7, 1234, 0)
    assert u[9] == np.float32(int(w[1]) >> 8) / np.float32(16777216.0)
    # step and salt give different streams
    assert not np.array_equal(u, dropout_uniform_ref(10001, 1234, 8, 1))
    assert not np.array_equal(u, dropout_uniform_ref(10001, 1234, 7, 0))


def test_dropout_seed_folds_into_int64():
    """TrainStep's default dropout seed is torch.initial_seed(), any 64-bit
    unsigned value; stack.device_dropout hands the op (an int64 schema
    argument) the same bit pattern as a signed value."""
    from spotv2net_amd.stack import _int64_seed
    for s in (0, 5154, 2 ** 63 - 1, 2 ** 63, 2 ** 63 + 5, 2 ** 64 - 1):
        v = _int64_seed(s)
        assert -2 ** 63 <= v < 2 ** 63
        assert v & 0xFFFFFFFFFFFFFFFF == s
