"""1x1 convolutions: graph-safe strided form and GEMM form.

Two modules replace ``nn.Conv2d`` 1x1 convolutions in place (same
parameters, state-dict keys and values):

* ``StridedConv1x1`` -- a strided 1x1 convolution as subsample + stride-1
  convolution (graph-safe, see below; the in-tree ResNets build their
  projection shortcuts with it);
* ``GemmConv1x1`` -- on channels_last activations, forward and ``dX`` as
  GEMMs on the NHWC activation matrix (fp32: the native bf16x3 GEMM,
  ``conv1x1_math``) and ``dW`` reduced in slabs
  (``_Conv1x1Gemm``); no MIOpen solver at all, and faster than MIOpen's 1x1
  solvers end to end (the bench default, ``bench.py --conv1x1``; required
  inside bf16 graphs, ``GraphedTrainStep(conv_mode='gemm')``).

Root cause of the whole-step graph corruption of rounds 2-3
(``profiles/graph_replay_r3_investigation.txt``; found with
``tools/graph_oop_audit.py`` / ``tools/graph_oop_bisect.py``, evidence in
``profiles/graph_oop_r4.md``): on MI355X, the HIP graph of MIOpen's
backward-data of a 1x1 convolution with stride 2 (ResNet's projection
shortcuts ``layer{2,3,4}.0.downsample.0``; fp32 and bf16, NHWC; a HIP memset
of ``dX`` followed by a composable-kernel ``grouped_conv_bwd_data`` launch)
reads device memory that neither the graph's private pool nor any live
tensor owns -- free blocks of the caching allocator's global pool.  Replays
are then correct only while nothing else writes those blocks: a second
model's eager steps, an eval pass or the K-FAC refresh step reuse them and
the shortcut's ``dX`` -- and every gradient upstream of it -- turns into
garbage or NaN.  Each of ResNet-50's 53 convolutions was captured alone and
replayed after every free global block was filled with 0xFF: only these
three changed, only in ``dX``, in fp32 and in bf16.

``StridedConv1x1`` computes the same convolution as a stride-1 1x1
convolution of the subsampled input, ``conv(x[:, :, ::s, ::s])``: identical
forward values, and a backward made of a stride-1 1x1 convolution (a GEMM in
MIOpen, graph-safe) plus the slice's scatter into a zero ``dX``.  The module
keeps ``stride == (s, s)``, its parameters and its state-dict keys, so K-FAC
sees exactly the layer it saw before (its hooks read the full-resolution
input and the module's stride) and checkpoints are unchanged.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from distributed_kfac_pytorch_amd.ops import _native as _nat
from distributed_kfac_pytorch_amd.utils.env import getenv

__all__ = ['StridedConv1x1', 'GemmConv1x1', 'ImplicitGemmConv2d', 'make_graph_safe',
           'is_strided_1x1', 'use_gemm_conv1x1', 'use_implicit_gemm_conv']


def is_strided_1x1(m: nn.Module) -> bool:
    """A 1x1, unpadded, undilated ``nn.Conv2d`` with a stride > 1."""
    return (
        isinstance(m, nn.Conv2d)
        and tuple(m.kernel_size) == (1, 1)
        and tuple(m.stride) != (1, 1)
        and m.padding in (0, (0, 0))
        and tuple(m.dilation) == (1, 1)
        and m.padding_mode == 'zeros'
    )


class _Subsample(torch.autograd.Function):
    """``x[:, :, ::sh, ::sw]`` as a channels_last tensor whose backward is
    ONE zero-fill + strided copy into a channels_last gradient.  Autograd's
    own slice backward builds two NCHW-contiguous zero tensors (one per
    sliced dim); the residual branch's channels_last gradient is then added
    to them by an unvectorised mixed-layout add -- 190 us for ResNet-50's
    layer2 input alone, ~0.5 ms per step over the three projection
    shortcuts (profiles/r5/prof_fp32_r6o/)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, sh: int, sw: int,  # type: ignore[override]
                slot: ResidualGradSlot | None = None) -> torch.Tensor:
        lib = _subsample_lib(x)
        ctx.conf = (x.shape, sh, sw, lib)
        ctx.slot = slot
        if lib is not None:  # csrc/subsample.hip: one 16-byte gather pass
            return lib.subsample_fwd(x, sh, sw)
        return x[:, :, ::sh, ::sw].contiguous(memory_format=torch.channels_last)

    @staticmethod
    def backward(ctx, g: torch.Tensor) -> tuple:  # type: ignore[override]
        shape, sh, sw, lib = ctx.conf
        g = g.contiguous(memory_format=torch.channels_last)
        slot = ctx.slot
        if slot is not None:
            base, slot.g, slot.done = slot.g, None, True
            if base is not None:
                # the block's other branch (conv1's input gradient, parked by
                # its backward): accumulate into it at the kept pixels only
                n, c, h, w = shape
                base = base.reshape(n, h, w, c).permute(0, 3, 1, 2)
                if lib is not None and base.is_contiguous(memory_format=torch.channels_last):
                    lib.subsample_bwd_acc(g, base, sh, sw)
                else:
                    base[:, :, ::sh, ::sw] += g
                return base, None, None, None
        if lib is not None:
            # one pass writing every element (a zero fill + strided copy ran
            # at 0.4 TB/s: 118 us at ResNet-50's layer2 input)
            return lib.subsample_bwd(g, shape[2], shape[3], sh, sw), None, None, None
        gx = g.new_zeros(shape).contiguous(memory_format=torch.channels_last)
        gx[:, :, ::sh, ::sw] = g
        return gx, None, None, None


def _subsample_lib(x: torch.Tensor):  # type: ignore[no-untyped-def]
    """The native library for fp32 CUDA channels_last tensors with C % 4 == 0."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.shape[1] % 4 == 0
            and x.data_ptr() % 16 == 0):
        return None
    return _nat.native()


def _subsample(x: torch.Tensor, sh: int, sw: int,
               slot: ResidualGradSlot | None = None) -> torch.Tensor:
    if x.is_contiguous(memory_format=torch.channels_last):
        if slot is not None:
            slot.armed = True
        return _Subsample.apply(x, sh, sw, slot)
    return x[:, :, ::sh, ::sw]


class StridedConv1x1(nn.Conv2d):
    """``nn.Conv2d`` (1x1, stride > 1) evaluated as subsample + stride-1
    conv (see the module docstring)."""

    def _conv_forward(  # type: ignore[override]
        self,
        input: torch.Tensor,
        weight: torch.Tensor,
        bias: torch.Tensor | None,
    ) -> torch.Tensor:
        sh, sw = self.stride
        sub = _subsample(input, sh, sw)
        return F.conv2d(sub, weight, bias, 1, 0, 1, self.groups)


def make_graph_safe(model: nn.Module, mode: str | None = None) -> int:
    """Make the 1x1 convolutions of ``model`` safe to capture (in place, same
    parameters).  Returns the number switched.

    ``mode`` (default ``KFAC_GRAPH_SAFE_CONV``, else ``strided``):

    * ``strided``: strided 1x1 convolutions become ``StridedConv1x1``; the
      stride-1 ones stay on MIOpen.  Besides the strided backward-data above,
      the tuned database's bf16 backward-weights solver of some stride-1 1x1
      shapes (``layer2.0.conv1``, ``layer2.2.conv3``: the assembly
      ``ConvAsmImplicitGemmGTCDynamicWrwXdlopsNHWC``, with a workspace) also
      read free global memory from a graph
      (profiles/graph_oop_r4/bisect_convs_bf16_tuned_db.jsonl).  Turning
      that solver off (``MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0``)
      is no cure: MIOpen then falls back to its naive direct kernels (fp32
      step 13x slower) and bf16's stem convolution is flagged instead
      (profiles/graph_oop_r4/bisect_convs_*_gtc_off.jsonl).  This mode is
      for fp32, whose replays match an eager twin bit for bit
      (tests/test_graphs_refresh_gpu.py).
    * ``gemm``: every 1x1 convolution becomes ``GemmConv1x1`` (hipBLASLt
      GEMMs, no MIOpen 1x1 solver in the graph at all) -- slower than MIOpen
      at the 56x56 stages (profiles/conv1x1_probe_r4.jsonl).
    """
    mode = mode or getenv('KFAC_GRAPH_SAFE_CONV', 'strided')
    if mode == 'gemm':
        return use_gemm_conv1x1(model)
    if mode != 'strided':
        raise ValueError(f'KFAC_GRAPH_SAFE_CONV={mode!r}: expected strided or gemm')
    n = 0
    for m in model.modules():
        if type(m) is nn.Conv2d and is_strided_1x1(m):
            m.__class__ = StridedConv1x1
            n += 1
    return n




# Knobs are read at call time through utils.env.getenv (~0.2 us a read, the
# eager step runs these paths ~100 times): a change of the environment takes
# effect on the next call, and two models in one process can differ.
def _slab_rows() -> int:
    return int(getenv('KFAC_CONV1X1_SLAB_ROWS', '2048'))


def _wgrad_1x1() -> str:
    return getenv('KFAC_CONV1X1_WGRAD', 'native')


def _wgrad_kxk() -> str:
    return getenv('KFAC_CONV_KXK_WGRAD', 'native')


def _conv_deterministic() -> bool:
    """``KFAC_CONV_DETERMINISTIC`` (default 1): the fp32 ``ImplicitGemmConv2d``
    backward keeps off MIOpen's nondeterministic solvers -- strided input
    gradients as ``dy . W`` plus a fixed-order col2im, 64-channel and stem
    weight gradients on the native split-K kernel -- so the fp32 step is bit
    reproducible (``tools/determinism_probe.py --fp32``)."""
    return getenv('KFAC_CONV_DETERMINISTIC', '1') == '1'


def _conv_deterministic_lowp() -> bool:
    """``KFAC_CONV_DETERMINISTIC_BF16`` (default 0, opt-in): under bf16
    autocast the ``ImplicitGemmConv2d`` / ``StemConv2d`` run as bf16 GEMMs
    (``_ConvLowpDet``: im2col forward, ``dy . W`` + the native bf16 col2im,
    ``dy^T . patches``) instead of MIOpen's bf16 solvers, whose global-split
    variants accumulate with atomics.  Not the default: it costs the bf16
    step ~2.5 ms (profiles/r6/deterministic_bf16/)."""
    return getenv('KFAC_CONV_DETERMINISTIC_BF16', '0') == '1'


def _splitk_few_tiles() -> bool:
    return getenv('KFAC_CONV1X1_SPLITK', '0') == '1'


def _bn_stats_on() -> bool:
    return getenv('KFAC_BN_CONV_STATS', '1') == '1'


# The BatchNorm statistics of a native convolution's output, written by the
# GEMM epilogue (csrc/gemm3.hip GemmDesc::bnpart), handed to the fused BN
# that consumes that output (ops/bnact.py bn_act): the convolution offers
# (its output tensor, the partials), the BN takes them if it was given that
# very tensor.  Only convolutions marked ``_feeds_bn`` (models/resnet.py)
# compute them.
_BN_SLOT: list = [None, None]


def _bn_part_for(m: int, n: int, device: torch.device) -> torch.Tensor:
    return torch.empty(2 * (-(-m // 128)) * 2 * n, device=device, dtype=torch.float32)


def _offer_bn_part(y: torch.Tensor, part: torch.Tensor | None) -> None:
    _BN_SLOT[0], _BN_SLOT[1] = (y, part) if part is not None else (None, None)


def take_bn_part(x: torch.Tensor) -> torch.Tensor | None:
    """The statistics partials of ``x`` if the native convolution that
    produced it offered them (cleared either way)."""
    y, part = _BN_SLOT
    if y is None:
        return None
    _BN_SLOT[0] = _BN_SLOT[1] = None
    return part if y is x else None


def _fuse_residual_grad() -> bool:
    return getenv('KFAC_RESIDUAL_GRAD_FUSE', '1') == '1'


class ResidualGradSlot:
    """Hand-off of an identity shortcut's gradient to the block's first
    1x1 convolution, whose input-gradient GEMM then adds it in its epilogue
    (csrc/gemm3.hip ``GemmDesc::D``) instead of autograd summing the two
    gradients of the block input with a separate add.

    ``_ResidualTap`` (the shortcut) runs its backward before the
    convolution's in the normal order (it is created after the block's last
    convolution, so the engine reaches it first) and parks its gradient
    here; if the convolution's backward ran first anyway, it marks ``done``
    and the tap returns its gradient to autograd as usual -- correct in
    either order."""

    __slots__ = ('g', 'done', 'armed')

    def __init__(self) -> None:
        self.g: torch.Tensor | None = None
        self.done = False
        self.armed = False


class _ResidualTap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, slot: ResidualGradSlot) -> torch.Tensor:  # type: ignore[override]
        ctx.slot = slot
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g: torch.Tensor) -> tuple:  # type: ignore[override]
        slot = ctx.slot
        if slot.done or g is None:
            return g, None
        slot.g = g
        return None, None


def residual_tap(x: torch.Tensor, slot: ResidualGradSlot) -> torch.Tensor:
    """The identity shortcut ``x`` whose gradient goes to ``slot``."""
    return _ResidualTap.apply(x, slot)


def conv1x1_math() -> str:
    """``KFAC_CONV1X1_MATH``: bf16x3 (default) or fp32 -- how an fp32
    ``GemmConv1x1`` computes its forward and input-gradient GEMMs.

    ``bf16x3``: the native grouped GEMM of csrc/gemm3.hip on one
    descriptor (``gemm3_mm``): each fp32 operand split into bf16 hi + lo on
    its way into LDS and multiplied as hi.hi + hi.lo + lo.hi on bf16 MFMA
    with fp32 accumulation -- relative error ~5e-6 against float64 (fp32
    hipBLASLt: 1e-7 - 1e-6; TF32, the reference's default for fp32
    convolutions on NVIDIA Ampere, ~1e-3).  On ResNet-50's stride-1 1x1
    shapes at batch 32 it takes 3.65 ms of forward + dX + dW per step
    against 4.97 ms for fp32 hipBLASLt (profiles/r5/conv1x1_gemm3_probe.jsonl),
    except where K >= 1024 leaves fewer than 128 output tiles (hipBLASLt's
    split-K wins there, and keeps those).  The weight gradient (K = N*H*W)
    runs split-K on the same kernel from 256 x 128 weights up
    (``_wgrad_native``, ``KFAC_CONV1X1_WGRAD=lib`` for hipBLASLt's slabs).  ``fp32``:
    hipBLASLt for everything (exact fp32 products, the A/B setting)."""
    return getenv('KFAC_CONV1X1_MATH', 'bf16x3').lower()


def _gemm3_lib(*ts: torch.Tensor, math: str | None = None):  # type: ignore[no-untyped-def]
    """The native library when the bf16x3 path (``math``, default
    ``conv1x1_math()``) applies to these operands."""
    if (not all(t.is_cuda and t.dtype == torch.float32 for t in ts)
            or (math or conv1x1_math()) != 'bf16x3'):
        return None
    return _nat.native()


def _gemm3_pays(m: int, n: int, k: int) -> bool:
    """bf16x3 tile GEMM vs hipBLASLt for C[m, n] with reduction k: the
    128 x 128 tiles lose to hipBLASLt's split-K only when a long reduction
    (k >= 1024) has fewer than 128 tiles to spread over 256 CUs."""
    tiles = -(-m // 128) * -(-n // 128)
    return k < 1024 or tiles >= 128


def _mm3(lib, a: torch.Tensor, b: torch.Tensor, n: int, b_kc: bool,  # type: ignore[no-untyped-def]
         bn: list | None = None, addend: torch.Tensor | None = None) -> torch.Tensor:
    """C[m, n] = a . B on gemm3_mm; split-K (fixed-order partial sum) when a
    long reduction leaves fewer than 128 tiles (``KFAC_CONV1X1_SPLITK=1``).
    ``bn``: a single pass also writes the output's BN statistics partials
    into ``bn[0]``.  ``addend``: C = a . B + addend, written into ``addend``."""
    m, k = a.shape
    tiles = -(-m // 128) * -(-n // 128)
    sp = 1
    if _splitk_few_tiles() and tiles < 128 and k >= 1024:
        sp = int(lib.gemm3_mm_splits(k, max(1, min(-(-256 // tiles), (k // 32) // 8))))
    if sp == 1:
        if addend is not None:
            lib.gemm3_mm(a, b, addend, True, b_kc, 1, None, addend)
            return addend
        y = torch.empty(m, n, device=a.device, dtype=a.dtype)
        part = _bn_part_for(m, n, a.device) if bn is not None else None
        lib.gemm3_mm(a, b, y, True, b_kc, 1, part)
        if bn is not None:
            bn[0] = part
        return y
    part = torch.empty(sp, m, n, device=a.device, dtype=a.dtype)
    lib.gemm3_mm(a, b, part, True, b_kc, sp)
    y = lib.sum_splits(part)
    return y if addend is None else y.add_(addend)


def _mm_nt(x: torch.Tensor, w: torch.Tensor, bn: list | None = None) -> torch.Tensor:
    """``x @ w.T`` for fp32 [m, k] x [n, k] (``bn``: as ``_mm3``)."""
    lib = _gemm3_lib(x, w)
    if lib is None or (not _splitk_few_tiles()
                       and not _gemm3_pays(x.shape[0], w.shape[0], x.shape[1])):
        return x @ w.t()
    return _mm3(lib, x, w, w.shape[0], True, bn)


def _mm_nn(g: torch.Tensor, w: torch.Tensor, addend: torch.Tensor | None = None) -> torch.Tensor:
    """``g @ w (+ addend)`` for fp32 [m, k] x [k, n]."""
    lib = _gemm3_lib(g, w)
    if lib is None or (not _splitk_few_tiles()
                       and not _gemm3_pays(g.shape[0], w.shape[1], g.shape[1])):
        return g @ w if addend is None else torch.addmm(addend, g, w)
    return _mm3(lib, g, w, w.shape[1], False, addend=addend)


def _splitk(m: int, rows: int | None = None) -> int:
    """Slabs of the weight-gradient reduction over ``m`` = N*H*W rows: the
    largest power of two that divides ``m`` and leaves >= ``rows`` rows each
    (``KFAC_CONV1X1_SLAB_ROWS``, default 2048)."""
    rows = rows or _slab_rows()
    s = 1
    while m % (2 * s) == 0 and m // (2 * s) >= rows:
        s *= 2
    return s


# blocks the split-K weight gradients aim for (KFAC_WGRAD_SPLIT_BLOCKS, also
# read by csrc/gemm3.hip gemm3_wgrad_splits): more splits fill the chip,
# fewer shrink the partial-sum pass


def _wgrad_native(lib, gy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:  # type: ignore[no-untyped-def]
    """``dW = dY^T X`` (fp32 [m, co] x [m, ci]) on the native bf16x3 GEMM
    with split-K over the m = N*H*W rows: ~512 blocks of >= 8 k-tiles
    each write fp32 partials, one fixed-order sum (deterministic)."""
    m, co = gy.shape
    ci = x.shape[1]
    tiles = -(-co // 128) * -(-ci // 128)
    want = max(1, min(-(-int(getenv('KFAC_WGRAD_SPLIT_BLOCKS', '512')) // tiles), (m // 32) // 8))
    sp = int(lib.gemm3_mm_splits(m, want))
    if sp == 1:
        gw = torch.empty(co, ci, device=gy.device, dtype=gy.dtype)
        lib.gemm3_mm(gy, x, gw, False, False)
        return gw
    part = torch.empty(sp, co, ci, device=gy.device, dtype=gy.dtype)
    lib.gemm3_mm(gy, x, part, False, False, sp)
    return lib.sum_splits(part)


class _Conv1x1Gemm(torch.autograd.Function):
    """``Y = X W^T (+ b)`` on the NHWC activation matrix, with the weight
    gradient ``dW = dY^T X`` reduced in slabs: one GEMM with K = N*H*W
    (100k rows at the 56x56 stage) leaves a 64x256 output to a handful of
    workgroups, while a batched GEMM over ``_splitk`` slabs plus a sum
    spreads it over the chip."""

    @staticmethod
    def forward(  # type: ignore[override]
        ctx, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, bn: list | None = None,
        slot: ResidualGradSlot | None = None, park: ResidualGradSlot | None = None,
    ) -> torch.Tensor:
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.slot = slot
        ctx.park = park
        if _gemm3_lib(x, w) is not None and x.stride(1) == 1 and w.is_contiguous():
            y = _mm_nt(x, w, bn if b is None else None)
            return y if b is None else y.add_(b)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy: torch.Tensor) -> tuple:  # type: ignore[override]
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            add = None
            slot = ctx.slot
            if slot is not None:
                # the identity shortcut's gradient (ResidualGradSlot), parked
                # by its tap: added in the GEMM epilogue, in place
                add, slot.g, slot.done = slot.g, None, True
                if add is not None:
                    if add.dim() == 4:  # an identity tap's [N, C, H, W] gradient
                        add = add.permute(0, 2, 3, 1)
                    add = add.reshape(x.shape)
                    if add.stride(1) != 1 or add.stride(0) != add.shape[1] or add.dtype != x.dtype:
                        add = add.contiguous().to(x.dtype)
            gx = _mm_nn(gy, w.contiguous(), add)
            park = ctx.park
            if park is not None and not park.done:
                # a projection block's conv1: the shortcut's backward (which
                # runs after this one) accumulates into this gradient
                park.g, gx = gx, None
        gw = None
        lib = _gemm3_lib(gy, x) if ctx.needs_input_grad[1] else None
        # native split-K from 256 x 128 weights up (51 vs 61 us there, 44 vs
        # 56-58 at 512 x 256 / 1024 x 512); hipBLASLt's slabs keep the small
        # 64-channel weights (37 vs 48 us): profiles/r5/conv1x1_gemm3_probe.jsonl
        if (lib is not None and _wgrad_1x1() == 'native'
                and gy.shape[1] * x.shape[1] >= int(getenv('KFAC_CONV1X1_WGRAD_MIN', '32768'))):
            gw = _wgrad_native(lib, gy, x)
        elif ctx.needs_input_grad[1]:
            m = gy.shape[0]
            s = _splitk(m)
            if s > 1:
                a, b = gy.view(s, m // s, -1).transpose(1, 2), x.view(s, m // s, -1)
                if gy.is_cuda and gy.dtype in (torch.bfloat16, torch.float16):
                    # fp32 slab partials (no per-slab rounding to 16 bits
                    # before the sum): hipBLASLt's fp32-output GEMM
                    part = torch.bmm(a, b, out_dtype=torch.float32)
                else:
                    part = torch.bmm(a, b)
                lib = _nat.native() if part.is_cuda and w.dtype == torch.float32 else None
                if lib is not None:
                    # fixed-order slab sum (csrc/subsample.hip sum_splits):
                    # one pass instead of torch's dim-0 reduction
                    gw = lib.sum_splits(part)
                else:
                    gw = part.sum(0, dtype=torch.promote_types(w.dtype, torch.float32)).to(w.dtype)
            else:
                gw = gy.t() @ x
        gb = gy.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb, None, None, None


class GemmConv1x1(StridedConv1x1):
    """``nn.Conv2d`` (1x1, unpadded, undilated, ungrouped, any stride) on
    channels_last activations evaluated as one GEMM:
    ``Y[NHW, Cout] = X[NHW, Cin] W[Cout, Cin]^T`` on the NHWC activation
    matrix (a strided conv first subsamples, as ``StridedConv1x1``).  The
    backward is ``dX = dY W`` and a slab-reduced ``dW = dY^T X``
    (``_Conv1x1Gemm``): in fp32 the forward and ``dX`` run on the native
    bf16x3 GEMM (``conv1x1_math``), the rest on hipBLASLt.  Same module,
    parameters and state-dict keys; other layouts or groups fall back to the
    convolution."""

    def _conv_forward(  # type: ignore[override]
        self,
        input: torch.Tensor,
        weight: torch.Tensor,
        bias: torch.Tensor | None,
    ) -> torch.Tensor:
        if self.groups != 1 or not input.is_contiguous(memory_format=torch.channels_last):
            return super()._conv_forward(input, weight, bias)
        sh, sw = self.stride
        x = input
        dev = x.device.type
        # the block's gradient hand-offs (models/resnet.py Bottleneck):
        # _dgrad_slot = add the slot's gradient to this input gradient,
        # _dgrad_park = park this input gradient for the shortcut
        slot = self.__dict__.pop('_dgrad_slot', None)
        park = self.__dict__.pop('_dgrad_park', None)
        if torch.is_autocast_enabled(dev):
            slot = park = None  # the gradients are summed by autograd
        if (sh, sw) != (1, 1):
            x = _subsample(input, sh, sw, slot)
            slot = park = None
        n, c, h, w = x.shape
        x2 = x.permute(0, 2, 3, 1).reshape(n * h * w, c)
        w2 = weight.view(weight.shape[0], c)
        if torch.is_autocast_enabled(dev):
            dt = torch.get_autocast_dtype(dev)
            x2, w2 = x2.to(dt), w2.to(dt)
            bias = bias.to(dt) if bias is not None else None
        bn = [None] if getattr(self, '_feeds_bn', False) and _bn_stats_on() else None
        for sl in (slot, park):
            if sl is not None:
                sl.armed = True
        with torch.autocast(dev, enabled=False):
            y = _Conv1x1Gemm.apply(x2, w2, bias, bn, slot, park)
        out = y.view(n, h, w, -1).permute(0, 3, 1, 2)
        if bn is not None:
            _offer_bn_part(out, bn[0])
        return out


def use_gemm_conv1x1(model: nn.Module) -> int:
    """Switch every 1x1 ``nn.Conv2d`` / ``StridedConv1x1`` of ``model`` (in
    place) to ``GemmConv1x1``.  Returns the number switched."""
    n = 0
    for m in model.modules():
        if (type(m) in (nn.Conv2d, StridedConv1x1) and tuple(m.kernel_size) == (1, 1)
                and m.padding in (0, (0, 0)) and tuple(m.dilation) == (1, 1)
                and m.groups == 1 and m.padding_mode == 'zeros'):
            m.__class__ = GemmConv1x1
            n += 1
    return n


def conv_kxk_math() -> str:
    """``KFAC_CONV_KXK_MATH``: bf16x3 (default) or fp32 -- how an fp32
    ``ImplicitGemmConv2d`` computes its forward and (stride 1) input
    gradient: the native implicit-GEMM convolution of csrc/gemm3.hip
    (patches gathered from the NHWC input on their way into LDS, bf16x3
    MFMA, ~5e-6 relative against float64) or MIOpen fp32."""
    return getenv('KFAC_CONV_KXK_MATH', 'bf16x3').lower()


class _ConvImplicit(torch.autograd.Function):
    """``y = conv2d(x, w, b, stride, pad)`` with the forward, the input
    gradient at stride 1 (the convolution of ``dy`` with the flipped,
    transposed kernel, read in place) and the weight gradient
    (``dy^T . patches(x)``, split-K) on the native implicit GEMM; strided
    input gradients as ``dy . W`` (gemm3) plus the native fixed-order col2im
    under ``KFAC_CONV_DETERMINISTIC`` (MIOpen's ``convolution_backward``
    otherwise, as for 64-channel weight gradients then).  ``miopen_fwd``:
    the forward through MIOpen (``StemConv2d``)."""

    @staticmethod
    def forward(  # type: ignore[override]
        ctx, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, stride: int, pad: int,
        lib,  # type: ignore[no-untyped-def]
        bn: list | None = None,
        miopen_fwd: bool = False,
    ) -> torch.Tensor:
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pad, b is not None, lib)
        if miopen_fwd:
            # the stem: MIOpen's forward is the faster one there, the
            # backward below is native
            return F.conv2d(x, w, b, stride, pad)
        xp = _pad4(x)
        part = None
        if bn is not None and b is None:
            n, c, h, wd = xp.shape
            k = w.shape[2]
            if int(lib.gemm3_conv_splits(n, h, wd, c, w.shape[0], k, w.shape[3], stride, pad)) == 1:
                ho = (h + 2 * pad - k) // stride + 1
                wo = (wd + 2 * pad - w.shape[3]) // stride + 1
                part = _bn_part_for(n * ho * wo, w.shape[0], x.device)
        y = lib.gemm3_conv(xp, _pad4(w).contiguous(memory_format=torch.channels_last),
                           stride, pad, False, part)
        if bn is not None:
            bn[0] = part
        if b is not None:
            y.add_(b.view(1, -1, 1, 1))
        return y

    @staticmethod
    def backward(ctx, gy: torch.Tensor) -> tuple:  # type: ignore[override]
        x, w = ctx.saved_tensors
        stride, pad, has_bias, lib = ctx.conf
        gy = gy.contiguous(memory_format=torch.channels_last)
        k = w.shape[2]
        gx = gw = gb = None
        native_dx = (ctx.needs_input_grad[0] and stride == 1 and k - 1 - pad >= 0
                     and w.shape[0] % 32 == 0 and x.shape[1] % 4 == 0)
        if native_dx:
            # the flipped, transposed kernel is read in place (flipw)
            gx = lib.gemm3_conv(gy, w.contiguous(memory_format=torch.channels_last), 1,
                                k - 1 - pad, True)
        det = _conv_deterministic()
        if (ctx.needs_input_grad[0] and not native_dx and det and stride > 1
                and x.shape[1] % 4 == 0):
            # strided: cols = dy . W ([pixels, Cout] x [Cout, kh*kw*C], the
            # channels_last weight read in place), then each input-gradient
            # element sums its taps in a fixed order (col2im)
            n, c, h, wd = x.shape
            cout = w.shape[0]
            w2 = w.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
            w2 = w2.reshape(cout, -1)
            cols = _mm3(lib, gy.permute(0, 2, 3, 1).reshape(-1, cout), w2, w2.shape[1], False)
            gx = lib.col2im_nhwc(cols, n, c, h, wd, k, w.shape[3], stride, pad)
        # native weight gradient (split-K over the pixels) from 128 input
        # channels up: 54-71 us vs MIOpen's 85-87; at 64 MIOpen's 85 beats
        # 96 (profiles/r5/conv3x3_probe.jsonl)
        # (the kernel indexes output pixels in 22 bits: larger inputs, e.g.
        # 128 channels at 512x512 from batch 16, go to MIOpen)
        native_dw = (ctx.needs_input_grad[1] and (x.shape[1] >= 128 or x.shape[1] < 4 or det)
                     and w.shape[0] % 4 == 0
                     and gy.shape[0] * gy.shape[2] * gy.shape[3] < (1 << 22)
                     and x.numel() + 4 * x.shape[0] * x.shape[2] * x.shape[3] < (1 << 31)
                     and _wgrad_kxk() == 'native')
        if native_dw:
            gw = lib.gemm3_conv_wgrad(_pad4(x), gy, k, w.shape[3], stride, pad)
            gw = gw[:, :x.shape[1]]
        mask = [ctx.needs_input_grad[0] and gx is None,
                ctx.needs_input_grad[1] and not native_dw, False]
        if any(mask):
            r = torch.ops.aten.convolution_backward(
                gy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1, mask)
            if mask[0]:
                gx = r[0]
            if mask[1]:
                gw = r[1]
        if has_bias and ctx.needs_input_grad[2]:
            gb = gy.sum((0, 2, 3))
        return gx, gw, gb, None, None, None, None, None


class _ConvLowpDet(torch.autograd.Function):
    """bf16 ``y = conv2d(x, w, b, stride, pad)`` (autocast off inside) as
    bf16 GEMMs with fp32 accumulation, bit-reproducible end to end: forward
    ``im2col(x) . W^T`` (the channels_last weight read as [Cout, kh*kw*C];
    MIOpen's tuned bf16 forward takes global-split solvers with atomics for
    the 512-channel 7x7-output convolutions), input gradient ``cols = dy .
    W`` then the native fixed-order col2im (C % 8 == 0; MIOpen otherwise),
    weight gradient ``dy^T . patches`` from the forward's saved patches."""

    @staticmethod
    def forward(  # type: ignore[override]
        ctx, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, stride: int, pad: int,
        lib,  # type: ignore[no-untyped-def]
    ) -> torch.Tensor:
        n, c, h, wd = x.shape
        cout, _, kh, kw = w.shape
        ho = (h + 2 * pad - kh) // stride + 1
        wo = (wd + 2 * pad - kw) // stride + 1
        patches = torch.empty(n * ho * wo, kh * kw * c, dtype=x.dtype, device=x.device)
        lib.im2col(x, patches, kh, kw, stride, stride, pad, pad, True)
        w2 = w.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(cout, -1)
        y2 = torch.mm(patches, w2.t()) if b is None else torch.addmm(b, patches, w2.t())
        ctx.save_for_backward(x, w, patches)
        ctx.conf = (stride, pad, b is not None, lib)
        return y2.view(n, ho, wo, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy: torch.Tensor) -> tuple:  # type: ignore[override]
        x, w, patches = ctx.saved_tensors
        stride, pad, has_bias, lib = ctx.conf
        gy = gy.contiguous(memory_format=torch.channels_last)
        n, c, h, wd = x.shape
        cout, _, kh, kw = w.shape
        gy2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            if c % 8 == 0:
                w2 = w.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
                cols = torch.mm(gy2, w2.reshape(cout, -1))
                gx = lib.col2im_nhwc(cols, n, c, h, wd, kh, kw, stride, pad)
            else:
                gx = torch.ops.aten.convolution_backward(
                    gy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                    [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            gw = torch.mm(gy2.t(), patches).view(cout, kh, kw, c).permute(0, 3, 1, 2)
        if has_bias and ctx.needs_input_grad[2]:
            gb = gy.float().sum((0, 2, 3)).to(gy.dtype)
        return gx, gw, gb, None, None, None


def _lowp_det_conv(m: nn.Conv2d, input: torch.Tensor, weight: torch.Tensor,
                   bias: torch.Tensor | None) -> torch.Tensor | None:
    """``_ConvLowpDet`` for a bf16-autocast convolution when
    ``KFAC_CONV_DETERMINISTIC_BF16`` applies, else None."""
    dev = input.device.type
    if (not input.is_cuda or not torch.is_autocast_enabled(dev)
            or torch.get_autocast_dtype(dev) != torch.bfloat16 or not _conv_deterministic_lowp()):
        return None
    lib = _nat.native()
    if lib is None:
        return None
    dt = torch.bfloat16
    x = input.to(dt).contiguous(memory_format=torch.channels_last)
    w = weight.to(dt)
    b = bias.to(dt) if bias is not None else None
    with torch.autocast(dev, enabled=False):
        return _ConvLowpDet.apply(x, w, b, m.stride[0], m.padding[0], lib)


def _pad4(t: torch.Tensor) -> torch.Tensor:
    """Zero-pad dim 1 (channels) of an NCHW-shaped tensor to a multiple of 4
    (the 3-channel stem: one pixel's channels = one float4), channels_last."""
    c = t.shape[1]
    if c % 4 == 0:
        return t
    if (t.is_cuda and t.dtype == torch.float32
            and t.is_contiguous(memory_format=torch.channels_last)):
        lib = _nat.native()
        if lib is not None:
            return lib.pad_channels4(t)  # one pass, no zero fill + cat
    z = t.new_zeros(t.shape[0], 4 - c % 4, *t.shape[2:])
    return torch.cat([t, z], 1).contiguous(memory_format=torch.channels_last)


def _implicit_shape_ok(m: nn.Conv2d) -> bool:
    kh, kw = m.kernel_size
    return (m.groups == 1 and tuple(m.dilation) == (1, 1) and m.padding_mode == 'zeros'
            and kh == kw and kh > 1 and isinstance(m.padding, tuple)
            and m.padding[0] == m.padding[1] and m.stride[0] == m.stride[1])


def _implicit_ok(m: nn.Conv2d) -> bool:
    # the 3-channel stem runs (4-channel padded) but slower than MIOpen's:
    # bench 1932 vs 1942-1950 img/s with it switched (it becomes a
    # StemConv2d: MIOpen forward, native weight gradient)
    return _implicit_shape_ok(m) and m.in_channels % 4 == 0


class ImplicitGemmConv2d(nn.Conv2d):
    """``nn.Conv2d`` (square kernel > 1, symmetric stride / padding, no
    groups or dilation: ResNet's 3x3 convolutions; a channel count that is
    not a multiple of 4 is zero-padded, but ``use_implicit_gemm_conv`` leaves
    the 3-channel stem to MIOpen, which is faster there) whose fp32
    channels_last forward and stride-1 input
    gradient run on the native implicit-GEMM kernel (``_ConvImplicit``,
    ``conv_kxk_math``; split-K over the 9 x C reduction when the image is
    too small to fill the chip).  ResNet-50 batch 32, per convolution:
    forward 58-71 us vs MIOpen fp32's 105-178 us at 128-512 channels, 84 vs
    90 us at 64 (profiles/r5/conv3x3_probe.jsonl); bench 1760 -> 1835 img/s
    with the 3x3 convolutions native.  Same module,
    parameters and state-dict keys (K-FAC sees an ``nn.Conv2d``); bf16
    autocast, other layouts and the CPU take ``nn.Conv2d``'s path."""

    def _conv_forward(  # type: ignore[override]
        self,
        input: torch.Tensor,
        weight: torch.Tensor,
        bias: torch.Tensor | None,
    ) -> torch.Tensor:
        y = _lowp_det_conv(self, input, weight, bias)
        if y is not None:
            return y
        lib = _gemm3_lib(input, weight, math=conv_kxk_math())
        if (lib is None or torch.is_autocast_enabled(input.device.type)
                or not input.is_contiguous(memory_format=torch.channels_last)):
            return super()._conv_forward(input, weight, bias)
        bn = [None] if getattr(self, '_feeds_bn', False) and _bn_stats_on() else None
        out = _ConvImplicit.apply(input, weight, bias, self.stride[0], self.padding[0], lib, bn)
        if bn is not None:
            _offer_bn_part(out, bn[0])
        return out


class StemConv2d(nn.Conv2d):
    """A convolution whose input channels are not a multiple of 4 (ResNet's
    3-channel stem): MIOpen's forward (faster there than the padded native
    one), and under ``KFAC_CONV_DETERMINISTIC`` the fp32 channels_last weight
    gradient on the native split-K kernel (``_ConvImplicit`` with
    ``miopen_fwd``) instead of MIOpen's global-split solver, whose atomics
    make it nondeterministic; the two cost the same
    (``tools/conv3x3_probe.py``, profiles/r6/).  Same module, parameters and
    state-dict keys as ``nn.Conv2d``."""

    def _conv_forward(  # type: ignore[override]
        self,
        input: torch.Tensor,
        weight: torch.Tensor,
        bias: torch.Tensor | None,
    ) -> torch.Tensor:
        y = _lowp_det_conv(self, input, weight, bias)
        if y is not None:
            return y
        lib = _gemm3_lib(input, weight, math=conv_kxk_math())
        if (lib is None or not _conv_deterministic()
                or torch.is_autocast_enabled(input.device.type)
                or not input.is_contiguous(memory_format=torch.channels_last)):
            return super()._conv_forward(input, weight, bias)
        return _ConvImplicit.apply(input, weight, bias, self.stride[0], self.padding[0], lib,
                                   None, True)


def use_implicit_gemm_conv(model: nn.Module) -> int:
    """Switch every eligible non-1x1 ``nn.Conv2d`` of ``model`` (in place)
    to ``ImplicitGemmConv2d`` (to ``StemConv2d`` when its input channels are
    not a multiple of 4).  Returns the number switched."""
    n = 0
    for m in model.modules():
        if type(m) is nn.Conv2d and _implicit_shape_ok(m):
            m.__class__ = ImplicitGemmConv2d if _implicit_ok(m) else StemConv2d
            n += 1
    return n

