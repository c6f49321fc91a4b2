import ctypes, torch, statistics, json, sys
sys.path.insert(0, '.')
from libfabric_amd import atomic
torch.cuda.set_device(0)
path = next(l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64.so' in l)
hip = ctypes.CDLL(path)
s = torch.cuda.current_stream()
for mib in (256, 32, 4):
    n = mib << 20
    nsets = max(4, (1 << 30) // (2 * n))
    sets = [(torch.empty(n, dtype=torch.uint8, device='cuda'), torch.randint(0, 255, (n,), dtype=torch.uint8, device='cuda')) for _ in range(nsets)]
    def memcpy(i):
        d, x = sets[i % nsets]
        assert hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_size_t(n), 3, ctypes.c_void_p(s.cuda_stream)) == 0
    def kern(i):
        d, x = sets[i % nsets]
        assert atomic.write_ptr(11, 1, d.data_ptr(), x.data_ptr(), n, s) == 0
    res = {}
    for name, fn in (('hipMemcpyAsync', memcpy), ('write_table_ATOMIC_WRITE', kern)):
        for i in range(20): fn(i)
        torch.cuda.synchronize()
        ts = []
        for r in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(40): fn(i)
            e1.record(s); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 40)
        t = statistics.median(ts)
        res[name] = {'us': round(t * 1e3, 2), 'frac': round(2 * n / (t * 1e-3) / 8e12, 4)}
    d, x = sets[0]; kern(0); torch.cuda.synchronize(); assert torch.equal(d, x)
    print(json.dumps({'mib': mib, **res}), flush=True)
