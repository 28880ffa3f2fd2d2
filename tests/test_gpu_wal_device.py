"""WAL recovery verify with the record chain walked on the device.

tkv_wal_verify copies the slurped image to HBM and tkv_wal_verify_device takes an image already
there; both walk the record_len chain of wal_entry::decode (/root/reference/src/engine/wal.cpp:63-130)
on the GPU in one sweep over the image (per-wave chunks, exact per-region walks, device-side fix-ups
where a chunk's speculative entry was wrong), check every record's CRC and report the first
corruption. No image is walked on the host. Every case is compared with a sequential decode written here
(header size, record_len, CRC via the test oracle, key/value bounds: wal.cpp:68-121), so the
parity is against the reference's decode order, not against the library's own host walk.
"""
import ctypes

import numpy as np
import pytest
import torch

import tinykvpp_amd as tk

pytestmark = pytest.mark.gpu


def sequential_decode(oracle, img, size):
    """wal_entry::decode applied record after record (engine.cpp:31-53 recovery loop)."""
    u32 = lambda p: int.from_bytes(img[p:p + 4].tobytes(), "little")  # noqa: E731
    recs, p, broke = [], 0, False
    while p < size:
        if size - p < 26:
            broke = True
            break
        rlen = u32(p)
        if rlen + 8 > size - p:
            broke = True
            break
        recs.append(p)
        p += 8 + rlen
    if recs:
        r = np.array(recs, np.uint64)
        rl = np.array([u32(int(x)) for x in r], np.uint64)
        got = oracle.batch(img, r + 8, rl.astype(np.uint32))
        stored = np.array([u32(int(x) + 4) for x in r], np.uint32)
        kv = np.array([26 + u32(int(x) + 18) + u32(int(x) + 22) <= 8 + int(l) for x, l in zip(r, rl)])
        bad = np.flatnonzero((got != stored) | ~kv)
        if bad.size:
            return "corrupted", int(bad[0]), int(r[bad[0]])
    return ("corrupted" if broke else "ok"), len(recs), p


def make_wal(rng, n_rec, vmax=16000, giant=(), fake_headers=0.0):
    """Stamped WAL image (numpy) of n_rec records laid out as wal.cpp:19-61. `giant`: record
    indices given 3-9 MiB values. fake_headers: fraction of values that embed a run of valid-looking
    records (speculative starts inside values)."""
    klen = rng.integers(0, 40, n_rec).astype(np.uint64)
    vlen = np.minimum(rng.zipf(1.6, n_rec) * 48, vmax).astype(np.uint64)
    for g in giant:
        vlen[g] = int(rng.integers(3 << 20, 9 << 20))
    size = 26 + klen + vlen
    offs = np.zeros(n_rec, np.uint64)
    offs[1:] = np.cumsum(size[:-1])
    img = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    hdr = np.zeros((n_rec, 26), np.uint8)
    hdr[:, 0:4] = (size - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 9:17] = np.arange(n_rec, dtype="<u8").view(np.uint8).reshape(-1, 8)
    hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(26)] = hdr
    if fake_headers:
        # values that hold a chain of well-formed 40-byte records: plausible headers off the chain
        fake = np.zeros(40, np.uint8)
        fake[0:4] = np.frombuffer((32).to_bytes(4, "little"), np.uint8)
        fake[18:22] = np.frombuffer((6).to_bytes(4, "little"), np.uint8)
        fake[22:26] = np.frombuffer((8).to_bytes(4, "little"), np.uint8)
        for i in np.flatnonzero(rng.random(n_rec) < fake_headers):
            v0, vl = int(offs[i] + 26 + klen[i]), int(vlen[i])
            reps = vl // 40
            if reps:
                img[v0:v0 + 40 * reps] = np.tile(fake, reps)
    lib = tk.load_library()
    size32 = size.astype(np.uint32)
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                               ctypes.c_void_p(size32.ctypes.data), n_rec))
    return img, offs, size


def wal_last():
    """What this thread's last WAL verify did (tkv_debug_wal_last): device rounds (the sweep plus its
    fix-up rounds), whether the exact host-thread walk had to finish it (only for a host image the
    device cannot hold), whether a host image was copied, whether the sweep needed no fix-up."""
    out = (ctypes.c_uint64 * 4)()
    tk.load_library().tkv_debug_wal_last(out)
    return {"passes": out[0], "host_walk": out[1], "copied": out[2], "fast": out[3]}


def wal_rounds():
    """Per fix-up round of this thread's last verify (tkv_debug_wal_rounds): failing boundaries, tasks,
    the longest task's range, all ranges, the most regions a task walked, all regions walked."""
    out = np.zeros(6 * 256, np.uint64)
    k = tk.load_library().tkv_debug_wal_rounds(ctypes.c_void_p(out.ctypes.data), out.size)
    keys = ("failing", "tasks", "longest", "regions", "walk_max", "walked")
    return [dict(zip(keys, map(int, out[i:i + 6]))) for i in range(0, min(k, out.size), 6)]


LAST = {}


def both(img, size, shift=0):
    """(host-image path, device-image path at byte offset `shift` of its allocation); LAST holds
    which path each took."""
    h = tk.wal.verify(img[:size].tobytes())
    LAST["host_image"] = wal_last()
    d = torch.zeros(size + shift, dtype=torch.uint8, device="cuda")
    if size:
        d[shift:] = torch.from_numpy(img[:size].copy()).cuda()
    dv = tk.wal.verify_device(d[shift:], size)
    torch.cuda.synchronize()
    LAST["device_image"] = wal_last()
    return h, dv


def device_walk_only(max_passes=1, fast=None):
    """Both verifies of the last `both` call finished on the device, in at most max_passes rounds
    (and, if `fast` is given, with or without fix-up rounds)."""
    for path, r in LAST.items():
        assert r["host_walk"] == 0, (path, r)
        assert 1 <= r["passes"] <= max_passes, (path, r)
        if fast is not None:
            assert r["fast"] == fast, (path, r)


@pytest.mark.parametrize("shift", [0, 3])
def test_small_records_clean_and_corrupted(gpu, oracle, shift):
    rng = np.random.default_rng(5)
    img, offs, size = make_wal(rng, 120000, vmax=600)
    n = img.size
    want = sequential_decode(oracle, img, n)
    assert want == ("ok", offs.size, n)
    assert both(img, n, shift) == (want, want)
    device_walk_only(fast=1)
    assert LAST["host_image"]["copied"] == 1 and LAST["device_image"]["copied"] == 0
    for bad in (0, 1, 777, 60000, 119999):  # payload flips: CRC mismatch at that record
        o = int(offs[bad]) + int(size[bad]) - 1
        img[o] ^= 0x01
        want = sequential_decode(oracle, img, n)
        assert want == ("corrupted", bad, int(offs[bad]))
        assert both(img, n, shift) == (want, want)
        device_walk_only()
        img[o] ^= 0x01


def test_giant_records_and_torn_tail(gpu, oracle):
    rng = np.random.default_rng(6)
    img, offs, size = make_wal(rng, 30000, giant=(10, 11, 20000, 29999))
    for n in (img.size, img.size - 5, int(offs[11]) + 30, int(offs[20000]) + 26 + 4096):
        want = sequential_decode(oracle, img, n)
        assert both(img, n) == (want, want), n
        print("giant records, n =", n, LAST)  # which path ran (passes, host walk)


def test_corrupted_record_len_and_overrun(gpu, oracle):
    """A record_len that lies sends the chain through garbage (the speculative pieces after it
    disagree, the walk resumes or stops exactly where the sequential decode does)."""
    rng = np.random.default_rng(7)
    img, offs, size = make_wal(rng, 50000, vmax=2000)
    n = img.size
    for bad, delta in ((100, 7), (25000, 4096), (49990, -3)):
        o = int(offs[bad])
        old = img[o:o + 4].copy()
        img[o:o + 4] = np.frombuffer((int(size[bad]) - 8 + delta).to_bytes(4, "little"), np.uint8)
        want = sequential_decode(oracle, img, n)
        assert want[0] == "corrupted" and want[1] == bad
        assert both(img, n) == (want, want)
        img[o:o + 4] = np.frombuffer((0xFFFFFF00).to_bytes(4, "little"), np.uint8)  # overruns the image
        want = sequential_decode(oracle, img, n)
        assert want == ("corrupted", bad, o)
        assert both(img, n) == (want, want)
        # the chain breaks with regions holding records after it: decided in the sweep, on the device
        device_walk_only(max_passes=8)
        img[o:o + 4] = old


def test_fake_headers_inside_values(gpu, oracle):
    """Values full of well-formed records: speculative starts land off the true chain and must be
    discarded by the stitch (exact result, clean and with a late corruption)."""
    rng = np.random.default_rng(8)
    img, offs, size = make_wal(rng, 40000, vmax=9000, fake_headers=0.5)
    n = img.size
    want = sequential_decode(oracle, img, n)
    assert want == ("ok", offs.size, n)
    assert both(img, n) == (want, want)
    print("fake headers, clean image:", LAST)  # which path ran: rounds, host walk
    device_walk_only(max_passes=10 ** 6)  # fix-up rounds, never the host walk
    o = int(offs[39000]) + 26
    img[o] ^= 0x80
    want = sequential_decode(oracle, img, n)
    assert both(img, n) == (want, want)
    print("fake headers, corrupted image:", LAST)
    device_walk_only(max_passes=10 ** 6)


@pytest.mark.parametrize("n", [0, 1, 25, 26, 27, 33, 34, 35, 255, 256, 257, 2047, 2048, 2049, 4096 + 17, 16383, 16384,
                               16385, 16384 + 1024 + 5])
def test_tiny_and_piece_boundary_images(gpu, oracle, n):
    rng = np.random.default_rng(9)
    img, offs, size = make_wal(rng, 400, vmax=200)
    want = sequential_decode(oracle, img, n)
    assert both(img, n) == (want, want)


def test_golden_records_on_device(gpu):
    from conftest import golden
    recs = [bytes.fromhex(r["hex"]) for r in golden("wal.json")["records"]]
    image = b"".join(recs)
    d = torch.frombuffer(bytearray(image), dtype=torch.uint8).cuda()
    assert tk.wal.verify_device(d) == ("ok", len(recs), len(image))
    bad = bytearray(image)
    bad[len(recs[0]) + 4] ^= 0xFF  # wal_test.cpp:809-850: parked at record 1
    d = torch.frombuffer(bad, dtype=torch.uint8).cuda()
    assert tk.wal.verify_device(d) == ("corrupted", 1, len(recs[0]))


def test_values_made_of_records(gpu, oracle):
    """Every value is itself a run of well-formed WAL records: chunk entries land on
    fake chains, and the device fix-ups settle the true chain without the host walk, clean and with a
    corruption near the end."""
    rng = np.random.default_rng(12)
    img, offs, size = make_wal(rng, 60000, vmax=4000, fake_headers=1.0)
    n = img.size
    want = sequential_decode(oracle, img, n)
    assert want == ("ok", offs.size, n)
    assert both(img, n) == (want, want)
    rounds = wal_rounds()
    print("values made of records:", LAST, rounds)
    device_walk_only(max_passes=10 ** 6)
    # bounded recovery: chunk entries settle within a few regions, a handful of
    # fix-up rounds, no fix-up task walks thousands of regions in sequence
    assert len(rounds) <= 4 and max(r["walk_max"] for r in rounds) <= 64, rounds
    o = int(offs[59000]) + 30
    img[o] ^= 0x40
    want = sequential_decode(oracle, img, n)
    assert both(img, n) == (want, want)
    device_walk_only(max_passes=10 ** 6)


def test_giant_values_made_of_records(gpu, oracle):
    """Forty 3-9 MiB values that are runs of well-formed records among 20 K record-valued records: chunk
    boundaries fall inside giant records whose hops are true, while the fake chains inside them hop on
    random record_len fields. Only a fake hop's fix-up task waits for its turn (kFakeHop): the device
    settles in a few rounds with no host walk and no task walking thousands of regions, clean and with a
    corruption past the giant records."""
    rng = np.random.default_rng(13)
    giant = tuple(int(g) for g in np.sort(rng.choice(np.arange(100, 19000), 40, replace=False)))
    img, offs, size = make_wal(rng, 20000, vmax=4000, giant=giant, fake_headers=1.0)
    n = img.size
    want = sequential_decode(oracle, img, n)
    assert want == ("ok", offs.size, n)
    assert both(img, n) == (want, want)
    rounds = wal_rounds()
    print("giant values made of records:", LAST, rounds)
    device_walk_only(max_passes=16)
    assert max(r["walk_max"] for r in rounds) <= 4096, rounds
    o = int(offs[19500]) + 30
    img[o] ^= 0x40
    want = sequential_decode(oracle, img, n)
    assert want[0] == "corrupted"
    assert both(img, n) == (want, want)
    device_walk_only(max_passes=16)


@pytest.mark.parametrize("plen", [0, 1, 17, 18, 239, 240, 241, 3000, 7168, 7200, 20000, 65536, 65537, 100000])
def test_payload_length_classes(gpu, oracle, plen):
    """Records whose payloads sit at the lane-fold limit (240 bytes) and past it (the long-payload
    batch), next to tiny corrupt ones (record_len < 18: key and value cannot fit)."""
    rng = np.random.default_rng(plen + 100)
    img, offs, size = make_wal(rng, 3000, vmax=300)
    n = img.size
    # rewrite record 1500 with a payload of plen bytes (record_len = plen), restamped
    recs = [img[int(offs[i]):int(offs[i]) + int(size[i])].tobytes() for i in range(offs.size)]
    klen = min(plen - 18, 4) if plen >= 18 else 0
    vlen = plen - 18 - klen if plen >= 18 else 0
    body = bytearray(rng.integers(0, 256, 26 + max(plen - 18, 0), dtype=np.uint8).tobytes())
    body[0:4] = plen.to_bytes(4, "little")
    body[8] = 0
    body[17] = 0
    body[18:22] = klen.to_bytes(4, "little")
    body[22:26] = vlen.to_bytes(4, "little")
    rec = bytes(body[:8 + plen]) if plen < 18 else bytes(body)
    recs[1500] = rec
    image = np.frombuffer(b"".join(recs), np.uint8).copy()
    offs2 = np.concatenate([[0], np.cumsum([len(r) for r in recs])[:-1]]).astype(np.uint64)
    sz2 = np.array([len(r) for r in recs], np.uint32)
    lib = tk.load_library()
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(image.ctypes.data), ctypes.c_void_p(offs2.ctypes.data),
                               ctypes.c_void_p(sz2.ctypes.data), offs2.size))
    m = image.size
    want = sequential_decode(oracle, image, m)
    assert both(image, m) == (want, want)
    if plen >= 18:
        assert want == ("ok", len(recs), m)
        o = int(offs2[1500]) + len(rec) - 1  # flip the record's last byte
        image[o] ^= 1
        want = sequential_decode(oracle, image, m)
        assert want[:2] == ("corrupted", 1500)
        assert both(image, m) == (want, want)
    else:
        assert want[:2] == ("corrupted", 1500)


REGION = 7168  # the sweep's region (tkv_wal_device.hip kRegion)


def record(rng, plen, klen=4):
    """One unstamped record with a payload of plen >= 18 bytes (wal.cpp:19-61 layout)."""
    vlen = plen - 18 - klen
    body = bytearray(rng.integers(0, 256, 26 + klen + vlen, dtype=np.uint8).tobytes())
    body[0:4] = plen.to_bytes(4, "little")
    body[4:8] = b"\0\0\0\0"
    body[8] = 0
    body[17] = 0
    body[18:22] = klen.to_bytes(4, "little")
    body[22:26] = vlen.to_bytes(4, "little")
    return bytes(body)


def region_end_records(rng):
    """Records (unstamped) placed so that long payloads sit at region ends: (records, [(index, start,
    payload length)] of the placed ones)."""
    lens = [241, 500, 4000, REGION - 8, REGION, REGION + 1, 15000, 30000, 65536]
    recs, pos, targets = [], 0, []
    for i, d in enumerate(list(range(0, 12)) + [26, 27, 100, 3000]):
        t = REGION * (4 + 12 * i) - d
        while t - pos > 3000:
            r = record(rng, int(rng.integers(22, 2000)))
            recs.append(r)
            pos += len(r)
        if t - pos < 30:
            t += REGION
            while t - pos > 3000:
                r = record(rng, int(rng.integers(22, 2000)))
                recs.append(r)
                pos += len(r)
        filler = record(rng, t - pos - 8)
        recs.append(filler)
        pos += len(filler)
        assert pos == t
        L = lens[i % len(lens)]
        if i % 3 == 2:  # the payload ends exactly on a region end
            L = (-(t + 8)) % REGION + REGION * (i % 4)
            L = max(L, 241) if L <= 65536 else 60000
        r = record(rng, L)
        targets.append((len(recs), pos, L))
        recs.append(r)
        pos += len(r)
    recs.append(record(rng, 100))
    return recs, targets


def test_long_payloads_at_region_ends(gpu, oracle):
    """Payloads of kLaneFold < record_len <= kMedMax are folded in the sweep's one read of the image:
    whole in a region, or carried across region ends (the register after the head, crc0 carries of the
    regions after, combined in wal_fin_*). Records placed so that their 8-byte prefix is cut by a region
    end (d = 1..8 bytes before it), their payload starts or ends exactly on one, and they span 1-10
    regions; clean, then each of a sample corrupted (first byte, last byte, a byte on a region end)."""
    rng = np.random.default_rng(77)
    recs, targets = region_end_records(rng)
    img = np.frombuffer(b"".join(recs), np.uint8).copy()
    offs = np.concatenate([[0], np.cumsum([len(r) for r in recs])[:-1]]).astype(np.uint64)
    sz = np.array([len(r) for r in recs], np.uint32)
    tk.check(tk.load_library().tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                             ctypes.c_void_p(sz.ctypes.data), offs.size))
    n = img.size
    want = sequential_decode(oracle, img, n)
    assert want == ("ok", len(recs), n)
    assert both(img, n) == (want, want)
    device_walk_only(max_passes=8)
    for idx, t, L in targets[::2]:
        a = t + 8
        for o in (a, a + L - 1, (a // REGION + 1) * REGION if (a // REGION + 1) * REGION < a + L else a + 1):
            img[o] ^= 0x10
            want = sequential_decode(oracle, img, n)
            assert want == ("corrupted", idx, t), (idx, t, L, o)
            assert both(img, n) == (want, want), (idx, t, L, o)
            img[o] ^= 0x10


def test_image_over_4_gib(gpu, oracle):
    """An image past 4 GiB (kPos32Max) takes the sweep's 64-bit positions (wal_sweep<*, uint64_t>):
    257 records of exactly 16 MiB (zero values: passed over and checked by the long-payload batch at
    offsets past 4 GiB), then 60 K Zipf records with 3-9 MiB values among them, all past 4 GiB. Clean,
    then a payload byte flipped in a small record past 4 GiB, in a giant record's value below it, and
    a torn tail: the verdict, good-record count and stop offset of wal.cpp:63-130 (the first bad
    record is the flipped one; every other record is stamped)."""
    rng = np.random.default_rng(44)
    big, nbig = 16 << 20, 257
    tail, toffs, tsize = make_wal(rng, 60_000, vmax=4000, giant=(100, 30_000))
    head = big * nbig
    size = head + tail.size
    assert size > 0xFFFF0000
    img = np.zeros(size, np.uint8)
    img[head:] = tail
    offs = np.arange(nbig, dtype=np.uint64) * big
    hdr = np.zeros((nbig, 26), np.uint8)
    hdr[:, 0:4] = np.full(nbig, big - 8, "<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 9:17] = np.arange(nbig, dtype="<u8").view(np.uint8).reshape(-1, 8)
    hdr[:, 22:26] = np.full(nbig, big - 26, "<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(26)] = hdr
    lib = tk.load_library()
    size32 = np.full(nbig, big, np.uint32)
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                               ctypes.c_void_p(size32.ctypes.data), nbig))
    for k in (0, nbig - 1):  # the stamp of two giant records against the oracle
        o = int(offs[k])
        assert oracle.crc(img[o + 8:o + big].tobytes()) == int.from_bytes(img[o + 4:o + 8].tobytes(), "little")
    nrec = nbig + toffs.size
    d = torch.from_numpy(img).cuda()
    del img
    assert tk.wal.verify_device(d, size) == ("ok", nrec, size)
    device_state = wal_last()
    assert device_state["host_walk"] == 0, device_state
    # a payload byte of tail record k (past 4 GiB), then of giant record 200's value (below 4 GiB)
    for pos, idx in ((head + int(toffs[777]) + 26 + 3, nbig + 777), (int(offs[200]) + 5000, 200)):
        d[pos] ^= 0x5A
        start = head + int(toffs[777]) if idx >= nbig else int(offs[200])
        assert tk.wal.verify_device(d, size) == ("corrupted", idx, start), pos
        d[pos] ^= 0x5A
    # a torn tail inside the last record
    cut = head + int(toffs[-1]) + 10
    assert tk.wal.verify_device(d, cut) == ("corrupted", nrec - 1, head + int(toffs[-1]))
    del d
    torch.cuda.empty_cache()
