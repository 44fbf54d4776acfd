"""Host side of the string directory: packing and the host mirror's id rule (first
occurrence, scramble_walk of the counter), with no GPU."""
import numpy as np

from distributedratelimiting.redis_amd.cluster import HostDirectory, scramble_walk
from distributedratelimiting.redis_amd.strdir import HostStringDirectory, pack_strings


def test_pack_strings():
    buf, offs = pack_strings(["ab", "", "héllo", b"\x00\x01"])
    assert offs.tolist() == [0, 2, 2, 8, 10]
    assert buf.size % 8 == 0 and bytes(buf[:10]) == b"ab" + "héllo".encode() + b"\x00\x01"


def test_first_occurrence_ids():
    h = HostStringDirectory(100)
    ids = h.assign(["b", "a", "b", "c"])
    ctr = scramble_walk(np.arange(3, dtype=np.uint64), 100)
    assert ids.tolist() == [ctr[0], ctr[1], ctr[0], ctr[2]]
    assert h.assign(["c", "d"]).tolist() == [ctr[2], scramble_walk(np.array([3], dtype=np.uint64), 100)[0]]
    assert h.lookup(["zz"]).tolist() == [2**64 - 1]


def test_same_rule_as_u64_directory():
    """Strings and u64 keys get ids by the same rule (both mirror tbe_hash.hpp)."""
    rng = np.random.default_rng(1)
    keys = rng.integers(0, 500, 2_000).astype(np.uint64)
    hs, hu = HostStringDirectory(1_000), HostDirectory(1_000)
    assert np.array_equal(hs.assign([str(k) for k in keys.tolist()]), hu.assign(keys))


def test_capacity_overflow():
    h = HostStringDirectory(3)
    ids = h.assign(["a", "b", "c", "d"])
    assert h.overflow and ids[3] == np.uint64(2**64 - 1)
