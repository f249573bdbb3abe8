import time, json, torch
torch.manual_seed(0)
dev = 'cuda'
res = {}
for n in (1024, 2304, 4608):
    x = torch.randn(n * 2, n, device=dev)
    a = (x.t() @ x) / (2 * n)
    for lib in ('default', 'magma'):
        try:
            torch.backends.cuda.preferred_linalg_library(lib)
            torch.linalg.eigh(a); torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(2):
                d, q = torch.linalg.eigh(a)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / 2 * 1e3
            err = ((q @ torch.diag(d) @ q.t() - a).abs().max() / a.abs().max()).item()
            print(json.dumps({'n': n, 'lib': lib, 'ms': round(ms, 2), 'recon_err': err}), flush=True)
        except Exception as e:
            print(json.dumps({'n': n, 'lib': lib, 'error': str(e)[:200]}), flush=True)
