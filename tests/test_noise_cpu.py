"""The noise generator's CPU restatement (oracle/philox_oracle.py) against the Random123 known-answer vectors
for philox4x32-10 (kat_vectors: counter, key -> output)."""
import philox_oracle as P

KAT = [  # ctr[4], key[2], expected[4]
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_kat():
    for ctr, key, want in KAT:
        assert P.philox4x32_10(ctr, key) == want


def test_uniform_mapping():
    u = P.uniform_noise(64, seed=0, draw=0)
    c = P.philox4x32_10((0, 0, 0, 0), (0, 0))
    assert abs(float(u[0]) - ((c[0] >> 8) * 2.0 ** -24 - 0.5)) == 0.0
    assert (u >= -0.5).all() and (u < 0.5).all()
