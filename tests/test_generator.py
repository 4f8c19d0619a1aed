"""CPU: the synthetic generator (host build) emits only frames the oracle
accepts, with the config's intended structure."""
import numpy as np
import pytest

import oracle as orc


@pytest.mark.parametrize("cfg,n", [("c1", 2000), ("c3", 3000), ("c4", 3000), ("c5", 4000),
                                   ("c6", 6000)])
def test_generated_frames_accepted(zp, cfg, n):
    arena, offs, lens = zp.batch.generate_host(cfg, n, first=12345)
    rec, _ = orc.parse_batch(arena, offs, lens)
    bad = np.nonzero(rec["err"])[0]
    assert len(bad) == 0, (bad[:5], rec["err"][bad[:5]])
    R = zp.records
    f = rec["flags"]
    if cfg == "c1":
        assert (lens == 64).all()
        assert ((f & R.F_UDP) != 0).all() and ((f & R.F_IPV4) != 0).all()
    if cfg == "c3":
        assert lens.min() >= 64 and lens.max() <= 1500
        assert ((f & R.F_IPV4) != 0).all()
        for b in (R.F_TCP, R.F_UDP, R.F_ICMPV4):
            assert 0.25 < ((f & b) != 0).mean() < 0.42
    if cfg == "c4":
        assert ((f & R.F_IPV6) != 0).all()
        assert 0.3 < ((f & R.F_EXT) != 0).mean() < 0.95
        assert (rec["eth_len"] == 22).any() and (rec["eth_len"] == 18).any()
    if cfg == "c5":
        assert set(np.unique(lens)) == {64, 576, 1500}
        assert 0.10 < ((f & R.F_IP_IN_IP) != 0).mean() < 0.3
        assert ((f & R.F_IP_IN_IP_V6) != 0).any()
    if cfg == "c6":
        # every header stack of c3-c5 plus ARP, mixed inside each 64-frame tile
        assert 0.03 < ((f & R.F_ARP) != 0).mean() < 0.10
        for b in (R.F_IPV4, R.F_IPV6, R.F_IP_IN_IP, R.F_EXT, R.F_TCP, R.F_UDP, R.F_ICMPV4,
                  R.F_ICMPV6):
            assert ((f & b) != 0).any(), b
        arp = (f & R.F_ARP) != 0
        assert (lens[arp] == 64).all() and set(np.unique(rec["eth_len"][arp])) == {14, 18, 22}
        tiles = f[: len(f) // 64 * 64].reshape(-1, 64)
        assert ((tiles & R.F_IPV4) != 0).any(1).all() and ((tiles & R.F_IPV6) != 0).any(1).all()
        assert ((tiles & R.F_ARP) != 0).any(1).mean() > 0.9


def test_generator_deterministic_per_packet(zp):
    a1, o1, l1 = zp.batch.generate_host("c5", 100, first=1000)
    a2, o2, l2 = zp.batch.generate_host("c5", 50, first=1050)
    for i in range(50):
        f1 = a1[o1[50 + i]:o1[50 + i] + l1[50 + i]]
        f2 = a2[o2[i]:o2[i] + l2[i]]
        assert f1.tobytes() == f2.tobytes()
