"""Per-batch counters (zp_stats_device): CPU checks of the
name table against the header, GPU checks against counts taken from the
oracle's records with numpy."""
import os
import re

import numpy as np
import pytest

import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def expected(rec):
    """The counters from oracle records (numpy): flag bits, then err codes."""
    flags = rec["flags"].astype(np.uint64)
    out = [int(((flags >> np.uint64(b)) & np.uint64(1)).sum()) for b in range(24)]
    out += list(np.bincount(rec["err"], minlength=38)[:38].astype(int))
    return np.array(out, np.int64)


def test_names_match_header(zp):
    h = open(os.path.join(ROOT, "include", "zero_packet.h")).read()
    assert int(re.search(r"#define ZP_STATS_FLAG_BITS (\d+)", h).group(1)) == zp.stats.FLAG_BITS
    assert zp.stats.COUNT == zp.stats.FLAG_BITS + len(zp.records.ERR_NAMES) == 62
    assert zp.stats.NAMES[6] == "tcp" and zp.stats.NAMES[12] == "ext:hop_by_hop"
    assert zp.stats.NAMES[24] == "err:OK" and zp.stats.NAMES[-1] == "err:OPTIONS_DATA_EXCEEDS"


def test_combine_sums_ranks(zp):
    a, b = np.arange(62), np.ones(62, np.int64)
    assert (zp.stats.combine([a, b]) == a + 1).all()


@pytest.mark.gpu
def test_stats_match_oracle(zp, golden):
    import torch
    from test_gpu_parity import fuzz_frames, pack
    d = torch.device("cuda:0")
    # a synthetic IMIX batch (ragged last wave) and a fuzz batch full of errors
    arena, offs, lens = zp.batch.generate("c5", 100_003, device=d)
    r, _ = zp.batch.parse_batch(arena, offs, lens)
    got = zp.stats.count(r)
    want = expected(orc.parse_batch(arena.cpu().numpy(), offs.cpu().numpy(),
                                    lens.cpu().numpy())[0])
    assert (got.cpu().numpy() == want).all()
    frames = fuzz_frames(zp, golden, 20000, 77)
    a, o, l_ = pack(frames)
    ta, to = torch.from_numpy(a).to(d), torch.from_numpy(o.astype(np.int64)).to(d)
    tl = torch.from_numpy(l_.astype(np.int32)).to(d)
    r2, _ = zp.batch.parse_batch(ta, to, tl)
    got2 = zp.stats.count(r2, counts=got)        # accumulates onto the first batch
    want2 = want + expected(orc.parse_batch(a, o, l_)[0])
    assert (got2.cpu().numpy() == want2).all()
    dct = zp.stats.to_dict(got2)
    assert dct["ethernet"] > 0 and sum(v for k, v in dct.items() if k.startswith("err:")) == \
        100_003 + len(frames)
    assert sum(v for k, v in dct.items() if k.startswith("err:") and k != "err:OK") > 1000


@pytest.mark.gpu
def test_stats_byte_counter_flush(zp):
    """48M synthetic records, 90 % of them with all 24 flag bits set: every
    lane runs past the 31 trips after which zp_stats_kernel flushes its SWAR
    byte counters (ST_GRID 512 x 256 lanes x ST_U 8 = 1M records per trip),
    and without that flush the byte counts (> 255 per lane) would carry into
    the next flag's byte. Counts equal numpy counts of the same records."""
    import torch
    d = torch.device("cuda:0")
    n = 48 << 20
    torch.manual_seed(5)
    full = torch.rand(n, device=d) < 0.9
    flags = torch.where(full, torch.full((n,), 0xFFFFFF, dtype=torch.int64, device=d),
                        torch.randint(0, 1 << 24, (n,), dtype=torch.int64, device=d))
    err = torch.where(torch.rand(n, device=d) < 0.8, torch.zeros(n, dtype=torch.int64, device=d),
                      torch.randint(0, 36, (n,), dtype=torch.int64, device=d))
    recs = torch.zeros((n, 8), dtype=torch.uint8, device=d)
    recs.view(torch.int32)[:, 0] = (flags | (err << 26)).to(torch.int32)   # err in bits 26-31
    got = zp.stats.count(recs).cpu().numpy()
    f = flags.cpu().numpy()
    want = [int(((f >> b) & 1).sum()) for b in range(24)]
    want += list(np.bincount(err.cpu().numpy(), minlength=38).astype(int))
    assert (got == np.array(want, np.int64)).all()
    assert got[0] > 40_000_000          # past the 8-bit range of one lane's byte counter


def test_count_refuses_bad_tensors(zp):
    """count() validates dtype and contiguity before the kernel writes
    counts (CPU tensors are refused first: no fallback)."""
    import torch
    with pytest.raises(RuntimeError):
        zp.stats.count(torch.zeros((4, 8), dtype=torch.uint8))


@pytest.mark.gpu
def test_count_refuses_bad_device_tensors(zp):
    import torch
    d = torch.device("cuda:0")
    with pytest.raises(ValueError):                      # int32 rows are not records
        zp.stats.count(torch.zeros((4, 4), dtype=torch.int32, device=d))
    big = torch.zeros((zp.stats.COUNT, 2), dtype=torch.int64, device=d)
    with pytest.raises(ValueError):                      # strided counts view
        zp.stats.count(torch.zeros((4, 8), dtype=torch.uint8, device=d), counts=big[:, 0])
    assert int(big.sum().item()) == 0
