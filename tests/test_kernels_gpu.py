"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32/fp64 math."""
from __future__ import annotations

import pytest
import torch

from distributed_kfac_pytorch_amd.ops import _native
from distributed_kfac_pytorch_amd.ops import comm_pack
from distributed_kfac_pytorch_amd.ops import factors
from distributed_kfac_pytorch_amd.ops import linalg
from distributed_kfac_pytorch_amd.ops import precondition as pops

pytestmark = pytest.mark.gpu


def _ref_cov(x: torch.Tensor, bias: bool) -> torch.Tensor:
    x = x.double()
    if bias:
        x = torch.cat([x, torch.ones(x.shape[0], 1, dtype=x.dtype, device=x.device)], 1)
    return x.t() @ x


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize(
    'n,k,bias',
    [
        (64, 10, False),
        (1000, 147, True),
        (4096, 256, False),
        (300, 129, True),
        (37, 520, False),
        (20000, 64, True),
        (512, 1152, False),
    ],
)
def test_syrk_matches_reference(cuda, dtype, n, k, bias):
    torch.manual_seed(0)
    x = torch.randn(n, k, device=cuda).to(dtype)
    d = k + int(bias)
    c0 = torch.randn(d, d, device=cuda)
    c0 = c0 + c0.t()
    for alpha, beta in ((1.0 / n, 0.0), (0.05 / n, 0.95)):
        out = c0.clone()
        factors.cov_accumulate_(out, x, bias=bias, alpha=alpha, beta=beta)
        ref = beta * c0.double() + alpha * _ref_cov(x, bias)
        err = (out.double() - ref).abs().max().item()
        scale = ref.abs().max().item()
        assert err <= 2e-5 * scale + 1e-6, (err, scale)
        # exact symmetry
        assert torch.equal(out, out.t())


def test_syrk_strided_rows(cuda):
    x = torch.randn(500, 200, device=cuda, dtype=torch.bfloat16)[:, :150]
    out = torch.empty(151, 151, device=cuda)
    factors.cov_accumulate_(out, x, bias=True, alpha=1.0, beta=0.0)
    ref = _ref_cov(x, True)
    assert (out.double() - ref).abs().max().item() < 1e-3 * ref.abs().max().item()


def test_syrk_split_k_forced(cuda):
    lib = _native.native()
    x = torch.randn(5000, 96, device=cuda)
    out = torch.zeros(96, 96, device=cuda)
    for splits in (1, 3, 17, 64):
        lib.syrk(x, out, False, 1.0, 0.0, splits)
        ref = _ref_cov(x, False)
        assert (out.double() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()
        assert torch.equal(out, out.t())


@pytest.mark.parametrize('d,bias', [(96, False), (147, True), (300, True)])
def test_syrk_split_k_deterministic_ema(cuda, d, bias):
    """The split-K workspace reduction sums partial tiles in a fixed order:
    repeated launches are bitwise identical, the EMA (beta) is applied once,
    and the result is exactly symmetric."""
    lib = _native.native()
    torch.manual_seed(1)
    k = d - int(bias)
    x = torch.randn(20000, k, device=cuda).to(torch.bfloat16)
    c0 = torch.randn(d, d, device=cuda)
    c0 = c0 + c0.t()
    outs = []
    for _ in range(3):
        out = c0.clone()
        lib.syrk(x, out, bias, 0.05 / x.shape[0], 0.95, 13)
        outs.append(out)
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    assert torch.equal(outs[0], outs[0].t())
    ref = 0.95 * c0.double() + (0.05 / x.shape[0]) * _ref_cov(x, bias)
    assert (outs[0].double() - ref).abs().max().item() < 2e-5 * ref.abs().max().item()
    assert lib.syrk_default_splits(20000, d) > 1


@pytest.mark.parametrize('natural', [True, False])
@pytest.mark.parametrize(
    'c,h,k,s,p',
    [(3, 17, 7, 2, 3), (16, 9, 3, 1, 1), (64, 8, 3, 2, 1), (8, 10, 1, 2, 0), (5, 6, 3, 1, 0)],
)
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_im2col(cuda, natural, c, h, k, s, p, dtype):
    x = torch.randn(2, c, h, h + 1, device=cuda).to(dtype)
    if natural:
        x = x.contiguous(memory_format=torch.channels_last)
    got, spatial = factors.conv_patches(x, (k, k), (s, s), (p, p), natural=natural)
    ref, spatial_ref = factors.conv_patches(
        x.cpu().float(), (k, k), (s, s), (p, p), natural=natural,
    )
    assert spatial == spatial_ref
    assert torch.equal(got.float().cpu(), ref.to(dtype).float())


@pytest.mark.parametrize('n', [1, 7, 64, 129, 300])
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_triu_roundtrip(cuda, n, dtype):
    a = torch.randn(n, n, device=cuda, dtype=dtype)
    a = a + a.t()
    packed = comm_pack.triu_pack(a)
    idx = torch.triu_indices(n, n, device=cuda)
    assert torch.equal(packed, a[idx[0], idx[1]])
    out = torch.empty_like(a)
    comm_pack.triu_unpack_(out, packed, 0.5)
    assert torch.allclose(out, 0.5 * a)


def _natural_patches(x: torch.Tensor, k, s, p) -> torch.Tensor:
    """Reference (kh, kw, c)-order patch matrix of an NCHW-logical input."""
    b, c, h, w = x.shape
    xp = torch.nn.functional.pad(x, (p[1], p[1], p[0], p[0]))
    u = xp.unfold(2, k[0], s[0]).unfold(3, k[1], s[1])  # [B, C, OH, OW, kh, kw]
    oh, ow = u.shape[2], u.shape[3]
    return u.permute(0, 2, 3, 4, 5, 1).reshape(b * oh * ow, k[0] * k[1] * c), oh * ow


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('cfg', [
    # (B, C, H, W, kernel, stride, padding, bias)
    (4, 16, 14, 14, (3, 3), (1, 1), (1, 1), False),
    (2, 64, 15, 13, (3, 3), (2, 2), (1, 1), True),
    (3, 32, 16, 16, (1, 1), (2, 2), (0, 0), False),
    (2, 8, 9, 11, (5, 3), (1, 2), (2, 0), True),
    (2, 136, 7, 7, (3, 3), (1, 1), (1, 1), False),
    # C % 8 != 0: fp32 takes the in-loop split staging, not the bf16 planes
    (2, 12, 10, 9, (3, 3), (1, 1), (1, 1), True),
    (3, 20, 8, 8, (3, 3), (2, 2), (1, 1), False),
])
def test_syrk_conv_implicit_im2col(cuda, cfg, dtype):
    if dtype == torch.bfloat16 and cfg[1] % 8:
        pytest.skip('bf16 implicit im2col needs C % 8 == 0 (explicit patches otherwise)')
    b, c, h, w, k, s, p, bias = cfg
    torch.manual_seed(sum(cfg[:4]))
    x = torch.randn(b, c, h, w, device=cuda).to(dtype).contiguous(
        memory_format=torch.channels_last)
    pm, spatial = _natural_patches(x.double(), k, s, p)
    if bias:
        pm = torch.cat([pm, pm.new_ones(pm.shape[0], 1)], 1)
    d = pm.shape[1]
    alpha, beta = 0.7 / pm.shape[0], 0.25
    c0 = torch.randn(d, d, device=cuda, dtype=torch.float64)
    c0 = (c0 + c0.t()).float()
    ref = beta * c0.double() + alpha * (pm.t() @ pm)
    out = c0.clone()
    assert factors.conv_cov_accumulate_(out, x, k, s, p, bias=bias, alpha=alpha, beta=beta)
    tol = 1e-5 if dtype == torch.float32 else 1e-4
    assert (out.double() - ref).abs().max().item() <= tol * ref.abs().max().item()
    assert torch.equal(out, out.t())


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
def test_syrk_conv_batch_slice(cuda, dtype):
    """A batch slice of a larger channels_last activation (the buffer-load
    range of the implicit im2col covers only the slice's extent)."""
    torch.manual_seed(3)
    full = torch.randn(6, 32, 12, 12, device=cuda).to(dtype).contiguous(
        memory_format=torch.channels_last)
    x = full[2:5]
    pm, _ = _natural_patches(x.double(), (3, 3), (1, 1), (1, 1))
    ref = pm.t() @ pm / pm.shape[0]
    out = torch.zeros(pm.shape[1], pm.shape[1], device=cuda)
    assert factors.conv_cov_accumulate_(out, x, (3, 3), (1, 1), (1, 1), alpha=1.0 / pm.shape[0])
    tol = 1e-5 if dtype == torch.float32 else 1e-4
    assert (out.double() - ref).abs().max().item() <= tol * ref.abs().max().item()


def test_syrk_conv_rejects_unaligned_channels(cuda):
    x = torch.randn(2, 3, 8, 8, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    out = torch.zeros(27, 27, device=cuda)
    assert not factors.conv_cov_accumulate_(out, x, (3, 3), (1, 1), (1, 1))


@pytest.mark.parametrize('n', [2, 10, 33, 64, 100, 128])
def test_jacobi_eigh(cuda, n):
    torch.manual_seed(n)
    b = 5
    x = torch.randn(b, n, 3 * n, device=cuda)
    a = x @ x.transpose(1, 2) / n
    evals, evecs = _native.native().jacobi_eigh(a.contiguous(), 15, 1e-7)
    ref = torch.linalg.eigvalsh(a.double())
    assert (evals.double() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()
    recon = evecs @ torch.diag_embed(evals) @ evecs.transpose(1, 2)
    assert (recon - a).abs().max().item() < 1e-4 * a.abs().max().item()
    eye = torch.eye(n, device=cuda).expand(b, n, n)
    assert (evecs.transpose(1, 2) @ evecs - eye).abs().max().item() < 1e-4
    # ascending
    assert bool((evals[:, 1:] >= evals[:, :-1]).all())


def test_eigh_many_mixed_sizes(cuda):
    mats = []
    for n in (3, 64, 64, 130, 200, 17):
        x = torch.randn(n, 2 * n, device=cuda)
        mats.append(x @ x.t() / n)
    res = linalg.eigh_many(mats)
    for m, (d, q) in zip(mats, res):
        recon = q @ torch.diag(d) @ q.t()
        assert (recon - m).abs().max().item() < 1e-4 * m.abs().max().item()


def test_eigh_many_rocsolver_sizes(cuda):
    """Mixed mid-size factors through the threaded chain lanes: the
    eigenpairs must match a float64 reference."""
    torch.manual_seed(3)
    mats = []
    for n in (512, 480, 440, 300, 260, 1024, 900):
        x = torch.randn(n, 2 * n, device=cuda)
        mats.append(x @ x.t() / (2 * n) + 1e-3 * torch.eye(n, device=cuda))
    res = linalg.eigh_many(mats)
    for m, (d, q) in zip(mats, res):
        n = m.shape[0]
        assert d.shape == (n,) and q.shape == (n, n)
        ref = torch.linalg.eigvalsh(m.double())
        assert (d.double() - ref).abs().max().item() < 1e-5 * ref.abs().max().item()
        recon = q @ torch.diag(d) @ q.t()
        assert (recon - m).abs().max().item() < 1e-5 * m.abs().max().item()
        eye = torch.eye(n, device=cuda)
        assert (q.t() @ q - eye).abs().max().item() < 1e-4


def _check_eigpairs(m, d, q, tol=2e-5):
    n = m.shape[0]
    ref = torch.linalg.eigvalsh(m.double())
    scale = ref.abs().max().item()
    assert (d.double() - ref).abs().max().item() < tol * scale
    recon = q.double() @ torch.diag(d.double()) @ q.double().t()
    assert (recon - m.double()).abs().max().item() < tol * scale
    eye = torch.eye(n, device=m.device, dtype=torch.float64)
    assert (q.double().t() @ q.double() - eye).abs().max().item() < 1e-4


def test_sytrd_reduce_reconstructs(cuda):
    """Native batched tridiagonalisation (csrc/sytrd.hip), mixed sizes in
    one chain: Q T Q^T must reproduce every input (Q formed on the host
    from the stored reflectors, float64)."""
    torch.manual_seed(5)
    sizes = (2, 3, 31, 32, 33, 65, 97)
    stacks, orig = [], []
    for n in sizes:
        x = torch.randn(2, n, n + 3, device=cuda)
        a = x @ x.transpose(1, 2) / n
        orig.append(a.clone())
        stacks.append(a.contiguous())
    flat = _native.native().sytrd_reduce(stacks)
    for s, (n, a0) in enumerate(zip(sizes, orig)):
        d, e, tau = flat[3 * s:3 * s + 3]
        for b in range(2):
            refl = stacks[s][b].double().cpu()
            qm = torch.eye(n, dtype=torch.float64)
            for k in range(n - 2, -1, -1):
                v = torch.zeros(n, dtype=torch.float64)
                v[k + 1] = 1.0
                v[k + 2:] = refl[k, k + 2:]
                qm = qm - float(tau[b, k]) * torch.outer(v, v @ qm)
            t = torch.diag(d[b].double().cpu())
            if n > 1:
                off = e[b, :n - 1].double().cpu()
                t = t + torch.diag(off, 1) + torch.diag(off, -1)
            recon = qm @ t @ qm.t()
            err = (recon - a0[b].double().cpu()).abs().max().item()
            assert err < 1e-5 * a0[b].abs().max().item(), (n, b, err)


@pytest.mark.parametrize('graphs', ['0', '1'])
@pytest.mark.parametrize('sizes', [(129, 130, 257, 300), (513, 1000, 64, 700, 2049)])
def test_eigh_many_sytrd_tier(cuda, monkeypatch, sizes, graphs):
    """eigh_many through the native sytrd tier (segmented chains, native
    divide and conquer, blocked UT back-transform), including rank-deficient
    K-FAC-like factors, vs a float64 reference; chain segments launched
    eagerly or replayed from captured HIP graphs."""
    monkeypatch.setenv('KFAC_SYTRD_GRAPHS', graphs)
    torch.manual_seed(7)
    # twice with the same sizes: the second refresh replays the chain's
    # captured HIP graphs on new matrices
    for rep in range(2):
        mats = []
        for j, n in enumerate(sizes):
            rows = n // 3 if (j + rep) % 2 else 2 * n  # rank-deficient PSD
            x = torch.randn(n, rows, device=cuda)
            mats.append(x @ x.t() / rows + 1e-3 * torch.eye(n, device=cuda))
        mats.append(mats[0].clone())  # duplicate size -> a bucket of 2
        res = linalg.eigh_many(mats)
        for m, (d, q) in zip(mats, res):
            assert d.shape == (m.shape[0],) and q.shape == m.shape
            _check_eigpairs(m, d, q)


@pytest.mark.parametrize('n', [1, 7, 64, 129, 176, 177, 300, 577, 640, 2049])
def test_spd_inverse(cuda, n):
    """K-HIP-5: blocked Cholesky damped inverses on fp32 MFMA tiles vs a
    float64 reference; exactly symmetric."""
    torch.manual_seed(n)
    b, damping = (3 if n < 1000 else 2), 1e-2
    x = torch.randn(b, n, 2 * n, device=cuda)
    f = x @ x.transpose(1, 2) / (2 * n)
    got = torch.stack(linalg.inverse_many(list(f), damping))
    eye = torch.eye(n, device=cuda, dtype=torch.float64)
    ref = torch.linalg.inv(f.double() + damping * eye)
    err = (got.double() - ref).abs().max().item()
    assert err < 2e-4 * ref.abs().max().item(), err
    assert torch.equal(got, got.transpose(1, 2))


def test_inverse_many_mixed(cuda):
    mats = []
    for n in (10, 10, 200, 33):
        x = torch.randn(n, 3 * n, device=cuda)
        mats.append(x @ x.t() / (3 * n))
    res = linalg.inverse_many(mats, 0.003)
    for m, inv in zip(mats, res):
        n = m.shape[0]
        ident = (m.double() + 0.003 * torch.eye(n, device=cuda, dtype=torch.float64)) @ inv.double()
        assert (ident - torch.eye(n, device=cuda, dtype=torch.float64)).abs().max().item() < 1e-3


def test_precondition_epilogues(cuda):
    g, a = 48, 97
    v = torch.randn(g, a, device=cuda)
    dgda = torch.rand(g, a, device=cuda)
    out = v.clone()
    pops.eigen_scale_(out, dgda=dgda)
    assert torch.allclose(out, v * dgda)
    dg, da = torch.rand(g, device=cuda), torch.rand(a, device=cuda)
    out = v.clone()
    pops.eigen_scale_(out, dg=dg, da=da, damping=0.01)
    assert torch.allclose(out, v / (torch.outer(dg, da) + 0.01), rtol=1e-5)

    p = torch.randn(g, a + 1, device=cuda)
    w = torch.randn(g, a, device=cuda)
    bvec = torch.randn(g, device=cuda)
    acc = torch.zeros(1, dtype=torch.float64, device=cuda)
    pops.kl_dot_(p, w, bvec, acc)
    ref = (p[:, :-1].double() * w.double()).sum() + (p[:, -1].double() * bvec.double()).sum()
    assert abs(acc.item() - ref.item()) < 1e-6 * abs(ref.item()) + 1e-6
    scale = torch.empty(1, device=cuda)
    pops.kl_finalize(acc, scale, 0.001, 0.1)
    vg = ref.item() * 0.01
    assert abs(scale.item() - min(1.0, (0.001 / abs(vg)) ** 0.5)) < 1e-6
    assert acc.item() == 0.0
    pops.apply_grad_(p, w, bvec, scale)
    assert torch.allclose(w, scale * p[:, :-1])
    assert torch.allclose(bvec, scale * p[:, -1])


def test_identity(cuda):
    c = torch.randn(70, 70, device=cuda)
    factors.identity_(c)
    assert torch.equal(c, torch.eye(70, device=cuda))


def _kfac_like(n: int, seed: int, cuda, drift: float = 0.02):
    """(old, new) K-FAC-like factors: EMA of batch covariances whose
    underlying basis drifts by a small rotation between the two."""
    g = torch.Generator().manual_seed(seed)
    lam = torch.exp(-torch.arange(n, dtype=torch.float64) / max(n / 8, 1.0))
    u, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    k = torch.randn(n, n, generator=g, dtype=torch.float64) * drift / n ** 0.5
    u2 = torch.linalg.matrix_exp(k - k.t()) @ u
    m = max(32, n // 2)

    def cov(b):
        x = (torch.randn(m, n, generator=g, dtype=torch.float64) * lam.sqrt()) @ b.t()
        return x.t() @ x / m

    a = torch.eye(n, dtype=torch.float64)
    for _ in range(12):
        a = 0.95 * a + 0.05 * cov(u)
    old = a.clone()
    for _ in range(10):
        a = 0.95 * a + 0.05 * cov(u2)
    return old.float().to(cuda), a.float().to(cuda)


def test_eigh_many_above_native_limit_falls_back(cuda, monkeypatch):
    """Factors above the native chain limit go to rocSOLVER's syevd (no
    host synchronisation), still exact."""
    monkeypatch.setattr(linalg, '_use_sytrd', lambda n: False)
    monkeypatch.setattr(linalg.twostage, 'max_n', lambda: 0)
    mats = []
    for j, n in enumerate((200, 333)):
        _, new = _kfac_like(n, 100 + j, cuda)
        mats.append(new)
    linalg.last_stats.clear()
    res = linalg.eigh_many(mats)
    assert {t[0] for t in linalg.last_stats['tiers']} == {'syevd'}, linalg.last_stats
    for m, (d, q) in zip(mats, res):
        _check_eigpairs(m, d, q)


@pytest.mark.parametrize('n', [177, 577, 2049])
def test_spd_inverse_rank_deficient_kfac(cuda, n):
    """Rank-deficient PSD factors (fewer rows than columns, as for the
    ResNet-50 layer4 A factors at batch 32) at the reference damping
    (condition number ~1e3-1e4): the blocked kernel is as accurate as the
    reference's fp32 routine (torch.linalg.inv, pivoted LU) against float64."""
    torch.manual_seed(n + 1)
    x = torch.randn(n // 3, n, device=cuda)
    f = (x.t() @ x / (n // 3)).contiguous()
    damping = 1e-3
    inv, fail = _native.native().spd_inverse_blocked(f.unsqueeze(0).contiguous(), damping)
    assert int(fail[0]) == 0
    eye = torch.eye(n, device=cuda)
    ref = torch.linalg.inv(f.double() + damping * eye.double())
    err = (inv[0].double() - ref).abs().max().item()
    lu32 = torch.linalg.inv(f + damping * eye)
    err_lu = (lu32.double() - ref).abs().max().item()
    assert err <= 4 * err_lu + 1e-6 * ref.abs().max().item(), (err, err_lu)


def test_inverse_many_indefinite_falls_back(cuda):
    """An indefinite 'damped factor' (e.g. a corrupted running average) makes
    the no-exchange elimination fail; inverse_many detects it on the device
    and re-solves with a pivoted LU: no NaN is installed."""
    for n in (40, 300):
        f = torch.eye(n, device=cuda)
        f[0, 0] = -1.0  # F + damping I is indefinite
        f[1, 1] = -0.5
        got = linalg.inverse_many([f], 0.01)[0]
        assert bool(torch.isfinite(got).all())
        ref = torch.linalg.inv(f.double() + 0.01 * torch.eye(n, device=cuda, dtype=torch.float64))
        assert (got.double() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('n,k,bias,splits', [
    (4096, 300, True, 0),    # default split-K
    (200, 130, False, 1),    # single split: the tile epilogue
    (50000, 64, True, 0),    # many splits, tiny D
    (777, 513, True, 3),
])
def test_syrk_packed_triangle_matches_dense(cuda, dtype, n, k, bias, splits):
    """The packed epilogue (factor all-reduce wire, parallel/comm.py
    PackedFactorBuffer) updates exactly the dense result's upper triangle."""
    torch.manual_seed(n + k)
    lib = _native.native()
    x = torch.randn(n, k, device=cuda).to(dtype)
    d = k + int(bias)
    c0 = torch.randn(d, d, device=cuda)
    c0 = (c0 + c0.t()) / 2
    alpha, beta = 0.3 / n, 0.9
    dense = c0.clone()
    lib.syrk(x, dense, bias, alpha, beta, splits)
    packed = comm_pack.triu_pack(c0)
    lib.syrk(x, packed, bias, alpha, beta, splits)
    # same accumulators; the epilogue's FMA contraction may differ by an ulp
    torch.testing.assert_close(packed, comm_pack.triu_pack(dense), rtol=1e-6, atol=1e-6)
    # through the factor op (1-D output selects the packed mode)
    p2 = comm_pack.triu_pack(c0)
    factors.cov_accumulate_(p2, x, bias=bias, alpha=alpha, beta=beta)
    p3 = comm_pack.triu_pack(c0)
    lib.syrk(x, p3, bias, alpha, beta, 0)  # the op uses the default split count
    assert torch.equal(p2, p3)


def test_syrk_conv_packed_triangle_matches_dense(cuda):
    torch.manual_seed(3)
    x = torch.randn(2, 136, 7, 7, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    d = 136 * 9 + 1
    c0 = torch.randn(d, d, device=cuda)
    c0 = (c0 + c0.t()) / 2
    dense = c0.clone()
    assert factors.conv_cov_accumulate_(dense, x, (3, 3), (1, 1), (1, 1), bias=True,
                                        alpha=0.01, beta=0.5)
    packed = comm_pack.triu_pack(c0)
    assert factors.conv_cov_accumulate_(packed, x, (3, 3), (1, 1), (1, 1), bias=True,
                                        alpha=0.01, beta=0.5)
    torch.testing.assert_close(packed, comm_pack.triu_pack(dense), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('exact', [False, True])
def test_syrk_fp32_input_modes(cuda, exact):
    """fp32 SYRK inputs: the default bf16x3 split (three bf16 MFMAs per
    fragment pair) stays within a few 1e-6 of the fp64 covariance; the
    exact-product fp32 MFMA mode within fp32 accumulation error."""
    torch.manual_seed(4)
    lib = _native.native()
    x = 3 * torch.randn(3000, 200, device=cuda)
    out = torch.empty(201, 201, device=cuda)
    lib.syrk(x, out, True, 1.0 / 3000, 0.0, 0, None, exact)
    ref = _ref_cov(x, True) / 3000
    rel = (out.double() - ref).abs().max().item() / ref.abs().max().item()
    assert rel < (2e-6 if exact else 1e-5), rel
    assert torch.equal(out, out.t())


@pytest.mark.parametrize('n,k,width,bias,splits', [
    (3000, 1024, 1024, True, 0),   # dense fp32, D >= 129, >= 2M elements: planes
    (4500, 512, 520, False, 3),    # strided rows, forced split-K
    (1100, 2048, 2048, True, 1),   # single split
    (1000, 512, 512, True, 0),     # below 2M elements: the in-loop split
    (9000, 256, 256, False, 0),    # two tiles
])
def test_syrk_dense_planes_fp32(cuda, n, k, width, bias, splits):
    """Dense fp32 SYRK inputs with D >= KFAC_SYRK_DENSE_PLANES_MIN_D (129)
    and >= 2M elements are split once into bf16 hi / lo planes and run on
    the planes kernel:
    fp32-class against fp64, exactly symmetric, bit-identical on repeat, and
    the packed-triangle output equals the dense one's upper triangle."""
    torch.manual_seed(n + k)
    lib = _native.native()
    x = (2 * torch.randn(n, width, device=cuda))[:, :k]
    d = k + int(bias)
    c0 = torch.randn(d, d, device=cuda)
    c0 = (c0 + c0.t()) / 2
    alpha, beta = 0.5 / n, 0.9
    outs = []
    for _ in range(2):
        out = c0.clone()
        lib.syrk(x, out, bias, alpha, beta, splits)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[0].t())
    ref = beta * c0.double() + alpha * _ref_cov(x, bias)
    rel = (outs[0].double() - ref).abs().max().item() / ref.abs().max().item()
    assert rel < 1e-5, rel
    packed = comm_pack.triu_pack(c0)
    lib.syrk(x, packed, bias, alpha, beta, splits)
    torch.testing.assert_close(packed, comm_pack.triu_pack(outs[0]), rtol=1e-6, atol=1e-6)


def test_eigh_many_repairs_nonfinite_results(cuda, monkeypatch):
    """A solver result with NaN (e.g. a divide-and-conquer failure that
    rocSOLVER reports only on the device) is detected and re-solved."""
    torch.manual_seed(13)
    mats = []
    for n in (200, 300):
        x = torch.randn(n, 2 * n, device=cuda)
        mats.append(x @ x.t() / (2 * n))
    real = linalg._launch_jobs

    def broken(gpu, stacks, dev, warms=None):
        res = real(gpu, stacks, dev, warms)
        k = sorted(res)[0]
        d, q = res[k]
        res[k] = (d, torch.full_like(q, float('nan')))
        return res

    monkeypatch.setattr(linalg, '_launch_jobs', broken)
    for m, (d, q) in zip(mats, linalg.eigh_many(mats)):
        assert torch.isfinite(q).all()
        _check_eigpairs(m, d, q)


@pytest.mark.parametrize('ta,tb', [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize('m,n,k,batch', [(128, 128, 16, 1), (100, 300, 77, 3), (512, 4608, 512, 2),
                                         (1, 65, 1000, 2), (257, 31, 2049, 1)])
def test_gemm_f32_matches_float64(cuda, ta, tb, m, n, k, batch) -> None:
    """csrc/gemm_f32.hip (the eigensolver's back-transform / D&C GEMMs) vs
    float64: exact fp32 products, fp32 accumulation."""
    lib = _native.native()
    g = torch.Generator(device='cpu').manual_seed(m + n + k)
    a = torch.randn(batch, *((k, m) if ta else (m, k)), generator=g)
    b = torch.randn(batch, *((n, k) if tb else (k, n)), generator=g)
    c0 = torch.randn(batch, m, n, generator=g)
    ref = 0.5 * (a.double().transpose(1, 2) if ta else a.double()) @ (
        b.double().transpose(1, 2) if tb else b.double()) - 2.0 * c0.double()
    c = c0.to(cuda)
    lib.gemm_f32(a.to(cuda), b.to(cuda), c, ta, tb, 0.5, -2.0)
    err = float((c.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 2e-6, err


def test_gemm_f32_strided_views(cuda) -> None:
    """Row-strided views (the in-place back-transform updates rows p+1.. of
    X with leading dimension n)."""
    lib = _native.native()
    x = torch.randn(2, 300, 300, device=cuda)
    v = torch.randn(2, 40, 300, device=cuda)[:, :, 17:]  # [2, 40, 283], row stride 300
    w = torch.randn(2, 40, 300, device=cuda)
    ref = x.double().clone()
    ref[:, 17:, :] -= v.double().transpose(1, 2) @ w.double()
    lib.gemm_f32(v, w, x[:, 17:, :], True, False, -1.0, 1.0)
    assert float((x.double() - ref).abs().max()) < 1e-4


@pytest.mark.parametrize('n,batch', [(1, 1), (64, 2), (200, 3), (512, 4), (511, 1)])
def test_trinv_upper_matches_float64(cuda, n, batch) -> None:
    """Blocked triangular inverse (64 x 64 back substitution + GEMM merges)
    of compact-WY-like upper-triangular matrices."""
    lib = _native.native()
    g = torch.Generator(device='cpu').manual_seed(n)
    u = torch.triu(torch.randn(batch, n, n, generator=g) * 0.1, diagonal=1)
    u = u + torch.diag_embed(1.0 + torch.rand(batch, n, generator=g))
    t = u.to(cuda).contiguous()
    lib.trinv_upper_(t)
    ref = torch.linalg.inv(u.double())
    err = float((t.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err
    assert torch.equal(torch.tril(t, diagonal=-1).cpu(), torch.zeros_like(u))
