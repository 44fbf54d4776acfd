"""Device string-key directory (include/tbe_strdir.h) against its
host mirror: InstanceName + resourceID -> dense id, exact strings (PTB:42).  Ids depend
only on first occurrence, so every case compares ids exactly."""
import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu


def _strings(rng, n, n_distinct, max_len=80):
    """n strings drawn from n_distinct random ones: random bytes (NUL included), lengths
    0..max_len, shared prefixes, some differing only in the last byte."""
    base = []
    for j in range(n_distinct):
        ln = int(rng.integers(0, max_len + 1))
        s = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
        if j % 7 == 3 and base:
            prev = base[-1]
            s = prev[:-1] + bytes([(prev[-1] + 1) % 256]) if prev else b"\x00"
        if j % 11 == 5:
            s = b"tenant/" + s
        base.append(s)
    base = list(dict.fromkeys(base))
    pick = rng.integers(0, len(base), n)
    return [base[k] for k in pick]


def _side_stream(gpu):
    import torch
    return torch.cuda.stream(torch.cuda.Stream(gpu))


def test_ids_match_host(engine_lib, gpu):
    from distributedratelimiting.redis_amd.strdir import HostStringDirectory, StringDirectory, to_device
    rng = np.random.default_rng(11)
    with _side_stream(gpu):
        d = StringDirectory(50_000, 4 << 20, prefix="api-gw-1:", device=0)
        h = HostStringDirectory(50_000)
        for b in range(4):
            s = _strings(rng, 20_000, 8_000)
            buf, offs, nb = to_device(s, gpu)
            ids = d.assign(buf, offs, nb).cpu().numpy().view(np.uint64)
            ref = h.assign(s)
            assert np.array_equal(ids, ref), b
        assert d.size() == h.size()
        # lookups: known strings, and strings never assigned
        s = _strings(rng, 5_000, 9_000) + [b"never-seen-1", b"never-seen-2" * 20]
        buf, offs, nb = to_device(s, gpu)
        got = d.lookup(buf, offs, nb).cpu().numpy().view(np.uint64)
        assert np.array_equal(got, h.lookup(s))
        assert d.size() == h.size()   # lookup assigns nothing


def test_long_and_empty_strings(engine_lib, gpu):
    from distributedratelimiting.redis_amd.strdir import HostStringDirectory, StringDirectory, to_device
    rng = np.random.default_rng(3)
    longs = [bytes(rng.integers(0, 256, 65536, dtype=np.uint8)), b"", b"a", b"a" * 65535]
    longs.append(longs[0][:-1] + bytes([longs[0][-1] ^ 1]))      # differs in the last byte only
    s = longs + longs[::-1] + [b""] * 3
    with _side_stream(gpu):
        d = StringDirectory(100, 1 << 20, device=0)
        h = HostStringDirectory(100)
        buf, offs, nb = to_device(s, gpu)
        assert np.array_equal(d.assign(buf, offs, nb).cpu().numpy().view(np.uint64), h.assign(s))
        for k in longs:
            assert d.key_of(int(h.lookup([k])[0])) == k


@pytest.mark.parametrize("bits", [14, 20])
def test_forced_hash_collisions(engine_lib, gpu, bits):
    """Hashes cut to `bits` bits: thousands of distinct strings share tags, so the byte
    comparison and the re-probe rounds decide; ids must not change."""
    from distributedratelimiting.redis_amd.strdir import HostStringDirectory, StringDirectory, to_device
    rng = np.random.default_rng(bits)
    with _side_stream(gpu):
        d = StringDirectory(20_000, 2 << 20, prefix="x", device=0, hash_bits=bits)
        h = HostStringDirectory(20_000)
        for b in range(3):
            s = [b"user-%d" % k for k in rng.integers(0, 6_000, 8_000)]
            buf, offs, nb = to_device(s, gpu)
            got = d.assign(buf, offs, nb).cpu().numpy().view(np.uint64)
            assert np.array_equal(got, h.assign(s)), b
        assert d.size() == h.size()
        s = [b"user-%d" % k for k in range(0, 7_000, 3)]
        buf, offs, nb = to_device(s, gpu)
        assert np.array_equal(d.lookup(buf, offs, nb).cpu().numpy().view(np.uint64), h.lookup(s))


def test_exhausted_rounds_report_erange(engine_lib, gpu):
    """4-bit hashes: 16 tags per round, 64 slots at most, so most of 200 strings cannot be
    placed.  Placed keys keep unique ids; the others get none; size() reports ERANGE."""
    from distributedratelimiting.redis_amd import _capi
    from distributedratelimiting.redis_amd.strdir import StringDirectory, to_device
    s = [b"k%d" % k for k in range(200)]
    with _side_stream(gpu):
        d = StringDirectory(1_000, 1 << 16, device=0, hash_bits=4)
        buf, offs, nb = to_device(s, gpu)
        ids = d.assign(buf, offs, nb).cpu().numpy().view(np.uint64)
        placed = ids[ids != np.uint64(2**64 - 1)]
        assert 0 < placed.size <= 64 and np.unique(placed).size == placed.size
        assert (placed < 1_000).all()
        with pytest.raises(_capi.TbeError) as ei:
            d.size()
        assert ei.value.status == _capi.TBE_ERANGE


def test_capacity_and_malformed(engine_lib, gpu):
    import torch
    from distributedratelimiting.redis_amd import _capi
    from distributedratelimiting.redis_amd.strdir import StringDirectory, to_device
    with _side_stream(gpu):
        d = StringDirectory(10, 1 << 12, device=0)
        s = [b"r%d" % k for k in range(25)]
        buf, offs, nb = to_device(s, gpu)
        ids = d.assign(buf, offs, nb).cpu().numpy().view(np.uint64)
        ok = ids[ids != np.uint64(2**64 - 1)]
        assert ok.size == 10 and np.array_equal(np.sort(ok), np.arange(10, dtype=np.uint64))
        with pytest.raises(_capi.TbeError) as ei:
            d.size()
        assert ei.value.status == _capi.TBE_ERANGE
        # malformed offsets (decreasing, past the buffer): no id, EINVAL state, no fault
        e = StringDirectory(10, 1 << 12, device=0)
        buf = torch.zeros(64, dtype=torch.uint8, device=gpu)
        offs = torch.tensor([0, 5, 3, 10, 10_000], dtype=torch.int64, device=gpu)
        ids = e.assign(buf, offs, 64).cpu().numpy().view(np.uint64)
        assert ids[1] == np.uint64(2**64 - 1) and ids[3] == np.uint64(2**64 - 1)
        assert ids[0] != np.uint64(2**64 - 1) and ids[2] != np.uint64(2**64 - 1)
        with pytest.raises(_capi.TbeError) as ei:
            e.size()
        assert ei.value.status == _capi.TBE_EINVAL


def test_host_buffer_entry(engine_lib, gpu):
    from distributedratelimiting.redis_amd.strdir import HostStringDirectory, StringDirectory
    rng = np.random.default_rng(5)
    d = StringDirectory(30_000, 2 << 20, device=0)
    h = HostStringDirectory(30_000)
    for b in range(2):
        s = _strings(rng, 10_000, 6_000, max_len=30)
        assert np.array_equal(d.assign_host(s), h.assign(s)), b


def test_strings_to_decisions(engine_lib, gpu):
    """The drop-in string path: resource strings -> device directory -> HIP engine, against
    the C restatement on the host mirror's ids (TB:202-238 per bucket string)."""
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    from distributedratelimiting.redis_amd.strdir import HostStringDirectory, StringDirectory, synthetic_key_text
    cap = 300_000
    rng = np.random.default_rng(8)
    with _side_stream(gpu):
        d = StringDirectory(cap, 16 << 20, prefix="svc:", device=0)
        h = HostStringDirectory(cap)
        eng = TokenBucketEngine(cap, 5, 2, 10_000_000, device=0)
        ref = cref.CTokenBucket(cap, 5, fill_rate(2, 10_000_000))
        for b in range(3):
            n = 100_000
            k = rng.zipf(1.3, n).astype(np.uint64) % np.uint64(200_000)
            buf, offs, nb = synthetic_key_text(torch.from_numpy(k.view(np.int64)).to(gpu), "user-")
            ids = d.assign(buf, offs, nb)
            p = rng.integers(0, 4, n).astype(np.int32)
            t = (1_760_000_000_000_000 + b * 700_000 + np.sort(rng.integers(0, 700_000, n))).astype(np.int64)
            g = torch.empty(n, dtype=torch.uint8, device=gpu)
            r = torch.empty(n, dtype=torch.int32, device=gpu)
            eng.acquire_batch_device(ids, torch.from_numpy(p).to(gpu), torch.from_numpy(t).to(gpu), g, r,
                                     stream=torch.cuda.current_stream(gpu).cuda_stream)
            hid = h.assign([b"user-%d" % v for v in k.tolist()])
            assert np.array_equal(ids.cpu().numpy().view(np.uint64), hid), b
            g_ref, r_ref = ref.acquire_batch(hid, p, t)
            assert np.array_equal(g.cpu().numpy(), g_ref) and np.array_equal(r.cpu().numpy(), r_ref), b


@pytest.mark.parametrize("mode", ["full", "warm", "auto"])
@pytest.mark.parametrize("hash_bits", [None, 22])
def test_assign_paths_match_host(engine_lib, gpu, mode, hash_bits):
    """The full pass, the warm path (lookup of the known strings, assign passes over the
    misses only) and the automatic choice give the host mirror's ids batch after batch:
    a cold batch, batches mostly known, a batch of only known strings, one of only new
    strings; with full hashes and with hashes cut to 22 bits (hundreds of shared tags, so
    misses re-probe, while no string collides in all four rounds)."""
    from distributedratelimiting.redis_amd.strdir import HostStringDirectory, StringDirectory, to_device
    rng = np.random.default_rng(5 + (hash_bits or 0))
    pool = [b"res/%06d/" % j + bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
            for j in range(50_000)]
    with _side_stream(gpu):
        d = StringDirectory(100_000, 8 << 20, prefix="gw:", device=0, hash_bits=hash_bits, mode=mode)
        h = HostStringDirectory(100_000)
        plan = [(0, 20_000), (0, 25_000), (0, 26_000), (0, 26_000), (30_000, 40_000), (0, 50_000)]
        for b, (lo, hi) in enumerate(plan):
            s = [pool[k] for k in rng.integers(lo, hi, 30_000)]
            buf, offs, nb = to_device(s, gpu)
            ids = d.assign(buf, offs, nb).cpu().numpy().view(np.uint64)
            assert np.array_equal(ids, h.assign(s)), (mode, b)
        assert d.size() == h.size()
        s = [pool[k] for k in rng.integers(0, 50_000, 5_000)]
        buf, offs, nb = to_device(s, gpu)
        assert np.array_equal(d.lookup(buf, offs, nb).cpu().numpy().view(np.uint64), h.lookup(s))
