"""Record codes (zp_set_record_slots, round 6): a full tile whose 64 records
all have the common form is stored by the parse kernel as one code byte per
frame and rewritten to its 64 records by zp_rec_expand_kernel. The records a
caller sees must be byte-identical to the oracle's and to the code-free
path's in every case: tiles with codes, tiles that lose them at the
checksum verdict, tiles of 64-B frames (the register path), ragged last
tiles, prior garbage in the records buffer, and the automatic mode at full
size."""
import ctypes
import os

import numpy as np
import pytest

import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_slot_mode_switch_cpu(built):
    """The switch is host state only (no GPU needed): returns the previous
    mode and refuses unknown ones."""
    lib = ctypes.CDLL(os.path.join(ROOT, "zero-packet_amd", "libzp_hip.so"))
    lib.zp_set_record_slots.argtypes = [ctypes.c_int]
    prev = lib.zp_set_record_slots(2)
    assert prev in (0, 1, 2)
    assert lib.zp_set_record_slots(1) == 2
    assert lib.zp_set_record_slots(3) == -1 and lib.zp_set_record_slots(-1) == -1
    assert lib.zp_set_record_slots(prev) == 1


# The code scheme restated on the host (zp_parse.hip rec_code / code_rec):
# the CPU tests below check its invariants on the oracle's own records, the
# GPU tests check that the kernels apply it.
F_ETH, F_ARP, F_V4, F_V6 = 1 << 0, 1 << 1, 1 << 2, 1 << 3
F_L4 = (0, 1 << 6, 1 << 7, 1 << 8, 1 << 9)              # none, TCP, UDP, ICMPv4, ICMPv6
CODE_BASE = 0xC0


def code_rec(c):
    x = c - CODE_BASE
    ec, l3, l4 = x // 15, x // 5 % 3, x % 5
    f = F_ETH | (F_ARP, F_V4, F_V6)[l3] | F_L4[l4] | ec << 24
    return f, (14 + 4 * ec + (20 if l3 == 1 else 40)) if l4 else 0


def rec_code(flags, offs):
    """The code of an ABI record, 0 if it has none (zp_parse.hip rec_code)."""
    for c in range(CODE_BASE, CODE_BASE + 45):
        x = c - CODE_BASE
        if x // 5 % 3 == 0 and x % 5:                  # ARP carries no L4 reader
            continue
        if code_rec(c) == (flags, offs):
            return c
    return 0


def test_code_scheme_bijective():
    """Every valid code names a distinct record whose byte 3 (err << 2 |
    Ethernet code) is below the 0xC0 marker, so a code tile can never be
    mistaken for records and the expansion is exact."""
    codes = [c for c in range(CODE_BASE, CODE_BASE + 45) if not (c - CODE_BASE) // 5 % 3 == 0
             or (c - CODE_BASE) % 5 == 0]
    assert len(codes) == 33                             # 3 Ethernet x (ARP + 2 x 5)
    recs = [code_rec(c) for c in codes]
    assert len(set(recs)) == len(codes)
    for c, (f, o) in zip(codes, recs):
        assert rec_code(f, o) == c and f >> 24 < 3
    assert (37 << 2 | 3) < CODE_BASE                    # any raw record's byte 3


@pytest.mark.parametrize("cfg", ["c1", "c2", "c3", "c4", "c5", "c6"])
def test_code_scheme_on_oracle_records(zp, cfg):
    """On each config's frames (and their truncations, for error records):
    a raw record's byte 3 stays below the marker, and a record with a code
    is exactly the record its code expands to, so the two stores agree."""
    a, o, l_ = zp.batch.generate_host(cfg, 1500, first=91)
    rng = np.random.default_rng(5)
    cut = l_.astype(np.int64)
    pick = rng.random(len(cut)) < 0.3
    cut[pick] = rng.integers(0, cut[pick] + 1)
    coded = 0
    for lens in (l_, cut.astype(np.uint32)):
        rec, ext = orc.parse_batch(a, o, lens)
        pk = orc.pack(rec, ext)
        assert (pk["flags"] >> 24 < CODE_BASE).all()
        for f, off in zip(pk["flags"].tolist(), pk["offs"].tolist()):
            c = rec_code(f, off)
            if c:
                coded += 1
                assert code_rec(c) == (f, off)
    if cfg in ("c1", "c2", "c3"):
        assert coded >= 1500                            # the common form is common here


torch = pytest.importorskip("torch")


def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


@pytest.fixture
def slots(zp):
    lib = zp._lib.hip()
    prev = lib.zp_set_record_slots(0)
    yield lambda mode: lib.zp_set_record_slots(mode)
    lib.zp_set_record_slots(prev)


def parse_modes(zp, slots, a, o, l_, fill=None):
    """Records under slots always (1) and never (2), as numpy (n, 8) bytes."""
    d = dev()
    at = torch.from_numpy(np.asarray(a, np.uint8)).to(d) if isinstance(a, np.ndarray) else a
    ot = torch.from_numpy(np.asarray(o, np.int64)).to(d) if isinstance(o, np.ndarray) else o
    lt = torch.from_numpy(np.asarray(l_, np.uint32).astype(np.int32)).to(d) \
        if isinstance(l_, np.ndarray) else l_
    out = {}
    for mode in (1, 2):
        slots(mode)
        n = ot.numel()
        rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
        rec.fill_(0xFF if fill is None else fill)
        ext = torch.zeros((2, n, 16), dtype=torch.uint8, device=d)
        r, e = zp.batch.parse_batch(at, ot, lt, rec, ext)
        torch.cuda.synchronize()
        out[mode] = zp.batch.records_to_numpy(r, e)
    return out


def check(zp, out, a, o, l_):
    want, wext = orc.parse_batch(np.asarray(a), np.asarray(o, np.uint64), np.asarray(l_, np.uint32))
    w = orc.pack(want, wext).view(np.uint8).reshape(-1, 8)
    for mode, (got, gext) in out.items():
        g = got.view(np.uint8).reshape(-1, 8)
        diff = np.nonzero((g != w).any(1))[0]
        assert len(diff) == 0, (mode, len(diff), diff[:5])
        assert zp.records.ext_match(gext, wext, want)
    return want


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n", [("c1", 64 * 200 + 5), ("c3", 64 * 400 + 63), ("c4", 64 * 300),
                                   ("c5", 64 * 500 + 1), ("c6", 64 * 400 + 30)])
def test_slots_configs_exact(zp, slots, cfg, n):
    arena, offs, lens = zp.batch.generate(cfg, n, first=777, device=dev())
    a, o, l_ = arena.cpu().numpy(), offs.cpu().numpy(), lens.cpu().numpy()
    out = parse_modes(zp, slots, arena, offs, lens)
    want = check(zp, out, a, o, l_)
    assert (want["err"] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("fill", [0x00, 0xFF, 0xA5])
def test_slots_verdict_changes_the_tile(zp, slots, fill):
    """c3 tiles built to reach every branch of the code decision: a tile
    whose walk records all have codes and whose verdict fails one frame's L4
    checksum (the records are stored after the verdict, without codes); a
    tile with an IPv4 header checksum error from the walk plus an L4 failure
    from the verdict and tiles with several walk errors (stored before the
    verdict); untouched tiles (codes). Any prior contents of the records
    buffer."""
    n = 64 * 64
    arena, offs, lens = zp.batch.generate("c3", n, first=31337, device=dev())
    a, o, l_ = arena.cpu().numpy().copy(), offs.cpu().numpy(), lens.cpu().numpy()
    rng = np.random.default_rng(3)
    for t in range(64):
        base = 64 * t
        kind = t % 4
        if kind == 1:                            # one L4 checksum failure
            i = base + int(rng.integers(0, 64))
            a[int(o[i]) + int(l_[i]) - 1] ^= 1
        elif kind == 2:                          # IPv4 header checksum + an L4 failure
            i, j = base + 3, base + 40
            a[int(o[i]) + 24] ^= 0x10             # header checksum byte
            a[int(o[j]) + int(l_[j]) - 1] ^= 2
        elif kind == 3:                          # many walk errors
            for k in range(6):
                i = base + 5 * k + 1
                a[int(o[i]) + [12, 14, 16, 22, 24, 47][k]] ^= 0x40
    out = parse_modes(zp, slots, a, o, l_, fill=fill)
    want = check(zp, out, a, o, l_)
    errs = want["err"].reshape(64, 64)
    assert (errs[1::4] != 0).sum(1).min() == 1
    assert all(len(np.unique(errs[t])) >= 3 for t in range(2, 64, 4))


@pytest.mark.gpu
def test_slots_min_size_tiles(zp, slots):
    """Tiles of 64-B frames take the register path, which stores codes too;
    a flipped bit sends its tile to the stream path."""
    n = 64 * 300 + 17
    arena, offs, lens = zp.batch.generate("c1", n, first=4, device=dev())
    a, o, l_ = arena.cpu().numpy().copy(), offs.cpu().numpy(), lens.cpu().numpy()
    rng = np.random.default_rng(9)
    for i in rng.choice(n, 40, replace=False):
        a[int(o[i]) + int(rng.integers(0, 64))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    out = parse_modes(zp, slots, a, o, l_)
    check(zp, out, a, o, l_)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_slots_auto_mode_full_size(zp, slots, cfg):
    """The automatic mode takes codes from 2,097,152 frames on, learning
    from probe calls whether the traffic has code tiles (c3: yes, c5: no):
    40 calls on 4M frames, back to back and with synchronisations between
    them (probes completing or not), each parse to the same bytes as the
    code-free path."""
    n = 4 << 20
    arena, offs, lens = zp.batch.generate(cfg, n, device=dev())
    slots(2)
    want = torch.full((n, 8), 0xFF, dtype=torch.uint8, device=arena.device)
    zp.batch.parse_batch(arena, offs, lens, want, check=False)
    slots(0)
    recs = [torch.full((n, 8), 0xA5, dtype=torch.uint8, device=arena.device) for _ in range(4)]
    for k in range(40):
        r = recs[k % 4]
        r.fill_(0xA5 if k % 2 else 0xFF)
        zp.batch.parse_batch(arena, offs, lens, r, check=False)
        if k % 3 == 0:
            torch.cuda.synchronize()
        if k % 4 == 3:
            torch.cuda.synchronize()
            for q in recs:
                assert torch.equal(q, want)
    assert int((zp.batch.record_err(want) != 0).sum()) == 0


@pytest.mark.gpu
def test_slots_mixed_tiles(zp, slots):
    """Config-5 tiles (IP-in-IP and VLAN tags: records) and config-3 tiles
    (codes) side by side in one batch, with one frame's L4 checksum failing
    in every third tile (those tiles store records after the verdict)."""
    a5, o5, l5 = zp.batch.generate_host("c5", 64 * 150, first=123)
    a3, o3, l3 = zp.batch.generate_host("c3", 64 * 150, first=456)
    frames = []
    for t in range(150):
        for a, o, l_ in ((a5, o5, l5), (a3, o3, l3)):
            frames += [bytearray(a[int(o[i]):int(o[i]) + int(l_[i])]) for i in range(64 * t, 64 * t + 64)]
    for t in range(0, 300, 3):
        f = frames[64 * t + 17]
        f[-1] ^= 1
    lens = np.array([len(f) for f in frames], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64))]).astype(np.int64)
    arena = np.zeros(int(offs[-1] + lens[-1]) + 64, np.uint8)
    for o, f in zip(offs, frames):
        arena[o:o + len(f)] = np.frombuffer(bytes(f), np.uint8)
    out = parse_modes(zp, slots, arena, offs, lens)
    want = check(zp, out, arena, offs, lens)
    inner = (want["flags"] & zp.records.F_IP_IN_IP) != 0
    assert inner.sum() > 1000 and (want["err"] != 0).sum() == 100


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_slots_auto_mode_under_graph_capture(zp, slots, cfg):
    """The automatic mode inside a HIP graph capture takes its last decision
    without probing (no event, no host word): the captured launches (the
    code kernels for c3 after a probe has run, the one-kernel path for c5)
    replay to the code-free path's records."""
    n = 4 << 20
    arena, offs, lens = zp.batch.generate(cfg, n, first=3, device=dev())
    slots(2)
    want = torch.empty((n, 8), dtype=torch.uint8, device=arena.device)
    zp.batch.parse_batch(arena, offs, lens, want, check=False)
    slots(0)
    warm = torch.empty((n, 8), dtype=torch.uint8, device=arena.device)
    for _ in range(3):                            # a probe, completed
        zp.batch.parse_batch(arena, offs, lens, warm, check=False)
        torch.cuda.synchronize()
    rec = torch.empty((n, 8), dtype=torch.uint8, device=arena.device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        zp.batch.parse_batch(arena, offs, lens, rec, check=False)
    for fill in (0x00, 0xFF):
        rec.fill_(fill)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(rec, want)
    assert torch.equal(warm, want)


@pytest.mark.gpu
def test_slots_auto_mode_threads(zp, slots):
    """zp_parse_batch_device in the automatic mode from four threads at once,
    each on its own stream with c3 (codes) and c5 (no codes) batches of 2M
    frames in turn: the per-device decision state is shared, the records
    are each batch's code-free records."""
    import threading
    n = 1 << 21
    d = dev()
    data = {cfg: zp.batch.generate(cfg, n, first=11, device=d) for cfg in ("c3", "c5")}
    slots(2)
    want = {}
    for cfg, (a, o, l_) in data.items():
        r = torch.empty((n, 8), dtype=torch.uint8, device=d)
        zp.batch.parse_batch(a, o, l_, r, check=False)
        want[cfg] = r
    torch.cuda.synchronize()
    slots(0)
    errors = []

    def work(k):
        try:
            s = torch.cuda.Stream(device=d)
            rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
            with torch.cuda.stream(s):
                for j in range(8):
                    cfg = ("c3", "c5")[(j + k) % 2]
                    a, o, l_ = data[cfg]
                    rec.fill_(0xA5)
                    zp.batch.parse_batch(a, o, l_, rec, check=False)
                    s.synchronize()
                    if not torch.equal(rec, want[cfg]):
                        errors.append((k, j, cfg))
        except Exception as e:                  # noqa: BLE001
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
