"""The numpy Philox restatement (tests/philox_ref.py) against the Random123 known-answer vectors
of philox4x32-10, and its subset order against a plain sort."""
import numpy as np

from philox_ref import philox, random_subset


def test_philox_known_answers():
    assert [int(v) for v in philox(np.uint64(0), 0, 0)] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    ones = 0xffffffffffffffff
    assert [int(v) for v in philox(np.uint64(ones), ones, ones)] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]


def test_subset_is_sorted_key_order():
    n, k = 300, 40
    x = philox(np.uint64(5) + np.arange(n, dtype=np.uint64), 2, 77)[0]
    ref = sorted(range(n), key=lambda i: (int(x[i]), i))[:k]
    assert random_subset(n, k, 77, 5, 2).tolist() == ref
