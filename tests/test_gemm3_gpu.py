"""Grouped bf16x3 GEMM (csrc/gemm3.hip) against fp64 PyTorch references."""
from __future__ import annotations

import copy

import pytest
import torch

import distributed_kfac_pytorch_amd as kfac
from distributed_kfac_pytorch_amd.ops import _native

pytestmark = pytest.mark.gpu


def _lib():
    lib = _native.native()
    assert lib is not None, _native.load_error()
    return lib


SHAPES = [  # M, N, K
    (64, 64, 64), (147, 2049, 37), (512, 4608, 256), (1000, 130, 2049),
    (33, 17, 5), (256, 1152, 128), (128, 128, 1),
]


@pytest.mark.parametrize('a_kc', [True, False])
@pytest.mark.parametrize('b_kc', [True, False])
def test_grouped_gemm_layouts(cuda, a_kc, b_kc):
    lib = _lib()
    torch.manual_seed(0)
    As, Bs, Cs, refs, extras, Ss, dgs, das, damps = [], [], [], [], [], [], [], [], []
    for i, (m, n, k) in enumerate(SHAPES):
        extra = a_kc and i % 2 == 1
        kmain = k - 1 if extra else k
        a_log = torch.randn(m, k, device=cuda)
        b_log = torch.randn(k, n, device=cuda)
        A = a_log[:, :kmain].contiguous() if a_kc else a_log.t().contiguous()
        ex = a_log[:, kmain].contiguous() if extra else None
        B = b_log.t().contiguous() if b_kc else b_log
        C = torch.full((m, n), float('nan'), device=cuda)
        ref = a_log.double() @ b_log.double()
        S = dg = da = None
        damp = 0.0
        if i % 3 == 1:
            S = torch.rand(m, n, device=cuda) + 0.5
            ref = ref * S.double()
        elif i % 3 == 2:
            dg = torch.rand(m, device=cuda)
            da = torch.rand(n, device=cuda)
            damp = 0.01
            ref = ref / (torch.outer(dg.double(), da.double()) + damp)
        As.append(A)
        Bs.append(B)
        Cs.append(C)
        refs.append(ref)
        extras.append(ex)
        Ss.append(S)
        dgs.append(dg)
        das.append(da)
        damps.append(damp)
    table, tiles, _ = lib.build_gemm_table(As, extras, Bs, Cs, Ss, dgs, das, damps, a_kc, b_kc)
    lib.gemm3_grouped(table, len(As), tiles, a_kc, b_kc)
    torch.cuda.synchronize()
    for (m, n, k), C, ref in zip(SHAPES, Cs, refs):
        assert torch.isfinite(C).all(), (m, n, k)
        err = (C.double() - ref).abs().max().item()
        # bf16x3: ~1e-5 relative per product (fp32 accumulation)
        assert err <= 5e-5 * ref.abs().max().item() + 1e-6, (m, n, k, err)


def test_grouped_gemm_strided_operands(cuda):
    """Row strides that are not multiples of 4 take the scalar load path."""
    lib = _lib()
    base_a = torch.randn(70, 133, device=cuda)
    base_b = torch.randn(131, 90, device=cuda)
    A = base_a[:, :129]      # lda 133
    B = base_b[:129, :77]    # ldb 90 (n-contig)
    C = torch.empty(70, 77, device=cuda)
    table, tiles, _ = lib.build_gemm_table([A], [None], [B], [C], [None], [None], [None], [0.0],
                                        True, False)
    lib.gemm3_grouped(table, 1, tiles, True, False)
    ref = A.double() @ B.double()
    assert (C.double() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()


def test_grouped_gemm_rejects_bad_shapes(cuda):
    lib = _lib()
    A = torch.randn(8, 8, device=cuda)
    B = torch.randn(9, 8, device=cuda)
    C = torch.empty(8, 8, device=cuda)
    with pytest.raises(RuntimeError):
        lib.build_gemm_table([A], [None], [B], [C], [None], [None], [None], [0.0], True, False)


def _convnet() -> torch.nn.Module:
    torch.manual_seed(0)
    return torch.nn.Sequential(
        torch.nn.Conv2d(3, 32, 3, padding=1),
        torch.nn.ReLU(),
        torch.nn.Conv2d(32, 64, 3, stride=2, bias=False),
        torch.nn.ReLU(),
        torch.nn.Conv2d(64, 130, 1),
        torch.nn.AdaptiveAvgPool2d(2),
        torch.nn.Flatten(),
        torch.nn.Linear(520, 37),
    )


@pytest.mark.parametrize('method', ['eigen', 'inverse'])
@pytest.mark.parametrize('prediv', [True, False])
@pytest.mark.parametrize('graphs', [True, False])
def test_grouped_precondition_matches_torch_chain(cuda, monkeypatch, method, prediv, graphs):
    base = _convnet().to(cuda).to(memory_format=torch.channels_last)
    models = [copy.deepcopy(base), copy.deepcopy(base)]
    pres = [
        kfac.KFACPreconditioner(
            m, factor_update_steps=1, inv_update_steps=3, compute_method=method,
            compute_eigenvalue_outer_product=prediv, lr=0.1,
        )
        for m in models
    ]
    if not graphs:
        for p in pres:
            p._graphs = None
    torch.manual_seed(3)
    for step in range(7):
        x = torch.randn(6, 3, 16, 16, device=cuda).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 37, (6,), device=cuda)
        grads = []
        for i, (m, p) in enumerate(zip(models, pres)):
            monkeypatch.setenv('KFAC_PRECOND_GEMM', 'bf16x3' if i == 0 else 'torch')
            for q in m.parameters():
                q.grad = torch.zeros_like(q) if q.grad is None else q.grad.zero_()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            p.step()
            grads.append([q.grad.clone() for q in m.parameters()])
        for a, b in zip(*grads):
            scale = b.abs().max().item()
            assert (a - b).abs().max().item() <= 1e-4 * scale + 1e-7, step
    assert pres[0]._grouped is not None and pres[0]._grouped._key is not None


@pytest.mark.parametrize('a_kc', [True, False])
@pytest.mark.parametrize('b_kc', [True, False])
def test_presplit_operands_bitwise_equal(cuda, a_kc, b_kc):
    """Pre-split bf16 hi/lo operands (eigenbases split once per update)
    give exactly the result of the in-kernel split."""
    lib = _lib()
    torch.manual_seed(4)
    shapes = [(64, 64, 64), (148, 2048, 36), (132, 96, 256), (36, 20, 8)]
    As, Bs, C1, C2, Ahl, Bhl = [], [], [], [], [], []
    for m, n, k in shapes:
        A = torch.randn(m, k, device=cuda) if a_kc else torch.randn(k, m, device=cuda)
        B = torch.randn(n, k, device=cuda) if b_kc else torch.randn(k, n, device=cuda)
        for X, out in ((A, Ahl), (B, Bhl)):
            r, c = X.shape
            hl = torch.empty((r, c // 4, 8), dtype=torch.bfloat16, device=cuda)
            xv = X.view(r, c // 4, 4)
            hl[:, :, :4].copy_(xv)
            hl[:, :, 4:].copy_(xv - hl[:, :, :4].float())
            out.append(hl)
        As.append(A)
        Bs.append(B)
        C1.append(torch.full((m, n), float('nan'), device=cuda))
        C2.append(torch.full((m, n), float('nan'), device=cuda))
    none = [None] * len(shapes)
    zeros = [0.0] * len(shapes)
    t1, n1, _ = lib.build_gemm_table(As, none, Bs, C1, none, none, none, zeros, a_kc, b_kc)
    lib.gemm3_grouped(t1, len(As), n1, a_kc, b_kc)
    t2, n2, _ = lib.build_gemm_table(As, none, Bs, C2, none, none, none, zeros, a_kc, b_kc,
                                     None, Ahl, Bhl)
    lib.gemm3_grouped(t2, len(As), n2, a_kc, b_kc)
    for c1, c2 in zip(C1, C2):
        assert torch.equal(c1, c2)


@pytest.mark.parametrize('method', ['eigen', 'inverse'])
@pytest.mark.parametrize('prediv', [False, True])
def test_split_grouped_matches_fp64_chain(cuda, monkeypatch, method, prediv):
    """KFAC_PRECOND_GEMM=split (pre-split images, LDS-DMA staged gemm3s):
    every step's preconditioned gradient P matches the fp64 chain computed
    from the SAME layer inputs (comparing two trajectories would measure the
    1/damping amplification of rounding noise, not the kernel)."""
    if method == 'inverse' and prediv:
        pytest.skip('prediv applies to the eigen method only')
    monkeypatch.setenv('KFAC_PRECOND_GEMM', 'split')
    torch.manual_seed(0)
    net = torch.nn.Sequential(
        torch.nn.Conv2d(3, 16, 3, padding=1, stride=2), torch.nn.ReLU(),
        torch.nn.Conv2d(16, 32, 3, bias=False), torch.nn.ReLU(), torch.nn.Flatten(),
        torch.nn.Linear(32 * 5 * 5, 130), torch.nn.ReLU(), torch.nn.Linear(130, 10),
    ).to(cuda)
    pre = kfac.KFACPreconditioner(
        net, factor_update_steps=1, inv_update_steps=2, compute_method=method,
        compute_eigenvalue_outer_product=prediv, lr=0.1, kl_clip=None)
    orig = pre._apply_gradients
    errs: list = []

    def check(ordered, kl):  # type: ignore[no-untyped-def]
        for _, l in ordered:
            wm = l.module.weight_grad_matrix().double()
            if l.module.has_bias():
                wm = torch.cat([wm, l.module.get_bias_grad().double()[:, None]], 1)
            if method == 'eigen':
                qa, qg = l.qa.double(), l.qg.double()
                v = qg.t() @ wm @ qa
                if l.dgda is not None:
                    v = v * l.dgda.double()
                else:
                    v = v / (torch.outer(l.dg.double(), l.da.double()) + pre.damping)
                ref = qg @ v @ qa.t()
            else:
                ref = l.g_inv.double() @ wm @ l.a_inv.double()
            errs.append(float((l.grad.double() - ref).abs().max() / ref.abs().max()))
        return orig(ordered, kl)

    pre._apply_gradients = check
    torch.manual_seed(1)
    for _ in range(5):
        x = torch.randn(16, 3, 14, 14, device=cuda)
        y = torch.randint(0, 10, (16,), device=cuda)
        net.zero_grad()
        torch.nn.functional.cross_entropy(net(x), y).backward()
        pre.step()
        with torch.no_grad():
            for p in net.parameters():
                p -= 0.05 * p.grad
    assert errs and max(errs) < 1e-4, errs
    g = pre._grouped
    assert type(g).__name__ == 'SplitGroupedPrecondition' and g._key is not None
