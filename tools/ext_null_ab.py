import ctypes, importlib, sys, torch
sys.path.insert(0, "/root/repo")
zp = importlib.import_module("zero-packet_amd")
d = torch.device("cuda:0")
n = 1 << 24
for cfg in ("c4", "c3"):
    arena, offs, lens = zp.batch.generate(cfg, n, device=d)
    rec = torch.empty((n, 8), dtype=torch.uint8, device=d)
    ext = torch.empty((2, n, 16), dtype=torch.uint8, device=d)
    lib = zp._lib.hip()
    s = torch.cuda.current_stream()
    res = {}
    for rnd in range(4):
        for name, e in (("ext", ext.data_ptr()), ("null", None)):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for a, b in ev:
                a.record(s)
                lib.zp_parse_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, rec.data_ptr(), e, ctypes.c_void_p(s.cuda_stream))
                b.record(s)
            torch.cuda.synchronize()
            res.setdefault(name, []).extend(a.elapsed_time(b) for a, b in ev)
    for k, v in res.items():
        v = sorted(v)
        print(cfg, k, round(v[len(v)//2], 4), flush=True)
    del arena, offs, lens, rec, ext
    torch.cuda.empty_cache()
