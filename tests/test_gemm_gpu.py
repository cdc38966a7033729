"""MFMA GEMM (csrc/gemm.hip) against plain PyTorch fp32 references, every operand
layout, both input dtypes, every epilogue, split-K; the wide-MLP op against autograd."""
import pytest
import torch

from distributed_training_pytorch_amd.models.wide import WideMLP
from distributed_training_pytorch_amd.ops import gemm as gemm_mod
from distributed_training_pytorch_amd.ops.gemm import colsum, gemm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ref(a, b, ta, tb):
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    return (A @ B.t()).float()


def _ops(M, N, K, ta, tb, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(*((K, M) if ta else (M, K)), generator=g).to(DEV, dtype)
    b = torch.randn(*((K, N) if tb else (N, K)), generator=g).to(DEV, dtype)
    return a, b


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(128, 128, 64), (200, 72, 40), (257, 300, 129), (64, 1, 10), (1, 37, 2)])
def test_gemm_f32_layouts(ta, tb, shape):
    M, N, K = shape
    a, b = _ops(M, N, K, ta, tb, torch.float32)
    c = gemm(a, b, trans_a=ta, trans_b=tb, splitk=1)
    torch.testing.assert_close(c, _ref(a, b, ta, tb), rtol=1e-5, atol=1e-4 * K ** 0.5)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(256, 256, 256), (200, 72, 40), (130, 520, 136), (64, 3, 8)])
def test_gemm_bf16_layouts(ta, tb, shape):
    M, N, K = shape
    a, b = _ops(M, N, K, ta, tb, torch.bfloat16)
    c = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32, splitk=1)
    # inputs are exact bf16 values: only the f32 accumulation order differs
    torch.testing.assert_close(c, _ref(a, b, ta, tb), rtol=1e-4, atol=1e-3 * K ** 0.5)
    cb = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, splitk=1)
    torch.testing.assert_close(cb.float(), c, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_gemm_bf16_big_tile_kernel(ta, tb):
    """>= 256 tiles of 256x256: the 32x32x16 MFMA kernel; ragged M/N edges, fused epilogue."""
    M, N, K = 8200, 4000, 320  # 33 x 16 = 528 tiles of 256x256
    a, b = _ops(M, N, K, ta, tb, torch.bfloat16, 7)
    bias = torch.randn(N, device=DEV)
    c = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32, splitk=1, bias=bias, force_big=True)
    ref = _ref(a, b, ta, tb) + bias
    torch.testing.assert_close(c, ref, rtol=1e-4, atol=2e-3 * K ** 0.5)
    cb = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, splitk=1, act=True, slope=0.1,
              force_big=True)
    torch.testing.assert_close(cb.float(), torch.nn.functional.leaky_relu(ref - bias, 0.1), rtol=1e-2, atol=5e-2)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(512, 768, 128), (1000, 1032, 320), (4104, 2056, 192), (1288, 776, 512)])
# default (8-phase by layout), two-buffer kernel, 8-phase balanced / unbalanced, 8-phase
# persistent tile walk (fast = 2 + variant; odd K-tile counts fall back to the unbalanced one)
@pytest.mark.parametrize("kernel", [True, 4, 34, 36, 37])
def test_gemm_bf16_fast_kernel(ta, tb, shape, kernel):
    """The LDS-DMA 256x256 kernel (row images + transposing LDS reads): every layout,
    ragged M/N edges, bias / LeakyReLU' (aux) epilogues, f32 and bf16 outputs."""
    M, N, K = shape
    a, b = _ops(M, N, K, ta, tb, torch.bfloat16, 11)
    bias = torch.randn(N, device=DEV)
    ref = _ref(a, b, ta, tb)
    c = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32, splitk=1, bias=bias, fast=kernel)
    torch.testing.assert_close(c, ref + bias, rtol=1e-4, atol=2e-3 * K ** 0.5)
    classic = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32, splitk=1, bias=bias, fast=False)
    torch.testing.assert_close(c, classic, rtol=1e-4, atol=2e-3 * K ** 0.5)
    aux = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    cb = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, aux=aux, slope=0.1, fast=kernel)
    torch.testing.assert_close(cb.float(), ref * torch.where(aux.float() > 0, 1.0, 0.1), rtol=1e-2, atol=5e-2)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("kernel", [True, 4, 34, 37])  # 8-phase default, two-buffer kernel, 8-phase balanced, persistent
def test_gemm_bf16_fast_kernel_accumulate_epilogues(ta, tb, kernel):
    """Epilogue operands of the LDS-DMA kernel: accumulate into f32 (the in-place weight
    gradient) and bf16 outputs, alpha + bias + LeakyReLU, and an output view whose rows
    are not 16-byte aligned (per-element path) next to the vector path."""
    M, N, K = 1000, 1032, 192
    a, b = _ops(M, N, K, ta, tb, torch.bfloat16, 13)
    ref = _ref(a, b, ta, tb)
    bias = torch.randn(N, device=DEV)
    old = torch.randn(M, N, device=DEV)
    c = gemm(a, b, trans_a=ta, trans_b=tb, out=old.clone(), accumulate=True, fast=kernel)
    torch.testing.assert_close(c, ref + old, rtol=1e-4, atol=2e-3 * K ** 0.5)
    oldb = old.to(torch.bfloat16)
    cb = gemm(a, b, trans_a=ta, trans_b=tb, out=oldb.clone(), accumulate=True, fast=kernel)
    torch.testing.assert_close(cb.float(), ref + oldb.float(), rtol=1e-2, atol=1e-1)
    ca = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, bias=bias, act=True, slope=0.1, alpha=0.5,
              fast=kernel)
    torch.testing.assert_close(ca.float(), torch.nn.functional.leaky_relu(0.5 * ref + bias, 0.1), rtol=1e-2, atol=5e-2)
    wide = torch.zeros(M, N + 3, device=DEV)
    view = wide[:, 3:]  # ld N + 3: rows not 16-byte aligned
    gemm(a, b, trans_a=ta, trans_b=tb, out=view, bias=bias, fast=kernel)
    torch.testing.assert_close(view, ref + bias, rtol=1e-4, atol=2e-3 * K ** 0.5)
    assert (wide[:, :3] == 0).all()


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("K", [1, 2, 13])
def test_gemm_skinny_k(ta, tb, K):
    """K <= 16 (first layer / last layer's input gradient): the output-bandwidth kernel,
    vector bf16 stores with bias, LeakyReLU'(aux) and LeakyReLU epilogues, ragged edges."""
    M, N = 1000, 1032
    a, b = _ops(M, N, K, ta, tb, torch.bfloat16, 5)
    bias = torch.randn(N, device=DEV)
    ref = _ref(a, b, ta, tb)
    c = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32, bias=bias, alpha=0.5)
    torch.testing.assert_close(c, 0.5 * ref + bias, rtol=1e-5, atol=1e-4)
    aux = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    cb = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, aux=aux, slope=0.1)
    torch.testing.assert_close(cb.float(), ref * torch.where(aux.float() > 0, 1.0, 0.1), rtol=1e-2, atol=2e-2)
    ca = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, bias=bias, act=True, slope=0.1)
    torch.testing.assert_close(ca.float(), torch.nn.functional.leaky_relu(ref + bias, 0.1), rtol=1e-2, atol=2e-2)
    af, bf = a.float(), b.float()
    cf = gemm(af, bf, trans_a=ta, trans_b=tb, bias=bias, act=True, slope=0.1)
    torch.testing.assert_close(cf, torch.nn.functional.leaky_relu(ref + bias, 0.1), rtol=1e-5, atol=1e-4)


def test_gemm_epilogues():
    M, N, K = 300, 200, 96
    a, b = _ops(M, N, K, False, False, torch.float32, 1)
    bias = torch.randn(N, device=DEV)
    aux = torch.randn(M, N, device=DEV)
    base = _ref(a, b, False, False)
    c = gemm(a, b, bias=bias, act=True, slope=0.1, alpha=0.5)
    torch.testing.assert_close(c, torch.nn.functional.leaky_relu(0.5 * base + bias, 0.1), rtol=1e-5, atol=1e-4)
    c = gemm(a, b, aux=aux, slope=0.01)
    torch.testing.assert_close(c, base * torch.where(aux > 0, 1.0, 0.01), rtol=1e-5, atol=1e-4)
    old = torch.randn(M, N, device=DEV)
    c = gemm(a, b, out=old.clone(), accumulate=True)
    torch.testing.assert_close(c, base + old, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("splitk", [2, 5])
def test_gemm_splitk(splitk):
    M, N, K = 96, 130, 1000
    a, b = _ops(M, N, K, True, True, torch.float32, 2)
    c = gemm(a, b, trans_a=True, trans_b=True, splitk=splitk)
    torch.testing.assert_close(c, _ref(a, b, True, True), rtol=1e-5, atol=1e-3)
    bias = torch.randn(N, device=DEV)
    c = gemm(a, b, trans_a=True, trans_b=True, splitk=splitk, bias=bias)
    torch.testing.assert_close(c, _ref(a, b, True, True) + bias, rtol=1e-5, atol=1e-3)


def test_gemm_strided_views():
    big = torch.randn(300, 512, device=DEV)
    a = big[:, 8:8 + 96]      # ld 512, offset: 16-byte aligned views stay vectorised
    b = torch.randn(64, 96, device=DEV)
    torch.testing.assert_close(gemm(a, b), _ref(a, b, False, False), rtol=1e-5, atol=1e-4)
    a2 = big[:, 3:3 + 96]     # misaligned: per-element fallback
    torch.testing.assert_close(gemm(a2, b), _ref(a2, b, False, False), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M", [5, 1000, 3000, 8195])
def test_colsum(M):
    x = torch.randn(M, 77, device=DEV)
    torch.testing.assert_close(colsum(x), x.sum(0), rtol=1e-5, atol=1e-4)
    out = torch.ones(77, device=DEV)
    torch.testing.assert_close(colsum(x.bfloat16(), out=out, accumulate=True), 1 + x.bfloat16().float().sum(0),
                               rtol=1e-4, atol=1e-3)
    xb = torch.randn(M, 264, device=DEV).bfloat16()  # N % 8 == 0: the 16-byte-load kernel
    torch.testing.assert_close(colsum(xb), xb.float().sum(0), rtol=1e-4, atol=1e-3)


def _emulated_forward(m, x, dtype):
    """The same graph in fp32 autograd, operands rounded to `dtype` where the kernels round them."""
    q = (lambda t: t.to(dtype).float()) if dtype != torch.float32 else (lambda t: t)
    lins = m.linears()
    h = q(x)
    for l, lin in enumerate(lins):
        z = h @ q(lin.weight).t() + lin.bias
        if l < len(lins) - 1:
            h = q(torch.nn.functional.leaky_relu(z, m.slope))
        else:
            h = z
    return h


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
def test_wide_mlp_grads_vs_autograd(dtype, tol):
    torch.manual_seed(0)
    m = WideMLP((2, 256, 192, 256, 1), compute_dtype=dtype).to(DEV)
    x = torch.randn(384, 2, device=DEV, requires_grad=True)
    y = torch.randn(384, 1, device=DEV)
    out = m(x)
    torch.nn.functional.mse_loss(out, y).backward()
    got = [p.grad.clone() for p in m.parameters()] + [x.grad.clone()]
    m.zero_grad()
    x.grad = None
    ref_out = _emulated_forward(m, x, dtype)
    torch.testing.assert_close(out, ref_out, rtol=tol, atol=tol)
    torch.nn.functional.mse_loss(ref_out, y).backward()
    ref = [p.grad for p in m.parameters()] + [x.grad]
    for g, r in zip(got, ref):
        rel = (g - r).abs().max() / r.abs().max().clamp_min(1e-6)
        assert rel < tol, rel


def test_toy_model_wide_width_runs_on_gemm_path():
    """ToyModel with hidden > 15 (no fused-kernel instance) trains through the MFMA GEMM:
    same forward / parameter gradients as its plain nn.Sequential twin."""
    from distributed_training_pytorch_amd.models.toy import ToyModel

    torch.manual_seed(3)
    m = ToyModel(hidden=96, depth=2).to(DEV)
    assert not m.uses_fused_kernel()
    x = torch.randn(300, 2, device=DEV)
    y = torch.randn(300, 1, device=DEV)
    torch.nn.functional.mse_loss(m(x), y).backward()
    got = [p.grad.clone() for p in m.parameters()]
    for p in m.parameters():
        p.grad = None
    torch.nn.functional.mse_loss(m.layers(x), y).backward()
    for g, p in zip(got, m.parameters()):
        torch.testing.assert_close(g, p.grad, rtol=1e-4, atol=1e-5)


def _wide_layer_cases(Bsz, W, slope=0.01):
    """The wide MLP's hidden-layer GEMMs with their epilogues: (kwargs, a, b, fp32 reference)."""
    g = torch.Generator().manual_seed(21)
    h = (torch.rand(Bsz, W, generator=g) * 2 - 1).to(DEV, torch.bfloat16)
    w = ((torch.rand(W, W, generator=g) * 2 - 1) / W ** 0.5).to(DEV, torch.bfloat16)
    dz = (torch.rand(Bsz, W, generator=g) * 2 - 1).to(DEV, torch.bfloat16)
    bias = torch.rand(W, generator=g).to(DEV) - 0.5
    old = torch.randn(W, W, generator=g).to(DEV)
    hf, wf, dzf = h.float(), w.float(), dz.float()
    return [
        ("fwd", dict(a=h, b=w, bias=bias, act=True, slope=slope, out_dtype=torch.bfloat16),
         torch.nn.functional.leaky_relu(hf @ wf.t() + bias, slope), 2e-2),
        ("last", dict(a=h, b=w, bias=bias, out_dtype=torch.float32), hf @ wf.t() + bias, 1e-3),
        ("dx", dict(a=dz, b=w, trans_b=True, aux=h, slope=slope, out_dtype=torch.bfloat16),
         (dzf @ wf) * torch.where(hf > 0, 1.0, slope), 2e-2),
        ("dx0", dict(a=dz, b=w, trans_b=True, out_dtype=torch.float32), dzf @ wf, 1e-3),
        ("dW", dict(a=dz, b=h, trans_a=True, trans_b=True, out=old.clone(), accumulate=True),
         dzf.t() @ hf + old, 1e-3),
    ]


def test_gemm_wide_layer_problems():
    """The wide-MLP layer problems (forward with bias + activation, last layer, dx with the
    activation gradient, dx of the first layer, dW accumulated) on the library's single
    backend, the HIP kernels."""
    for name, kw, ref, tol in _wide_layer_cases(2048, 1024):
        a, b = kw.pop("a"), kw.pop("b")
        got = gemm(a, b, **kw)
        rel = (got.float() - ref).abs().max() / ref.abs().max()
        assert rel < tol, (name, rel.item())


@pytest.mark.parametrize("M,N", [(1032, 2), (1, 1032), (3, 520), (2048, 4)])
@pytest.mark.parametrize("K", [300, 8200])
def test_gemm_skinny_output_weight_grad(M, N, K):
    """dW of an MLP's first / last Linear (min(M, N) <= 4, both operands K-major): the
    bandwidth kernel over the wide operand, fresh output, accumulate, alpha."""
    a, b = _ops(M, N, K, True, True, torch.bfloat16, 17)
    ref = _ref(a, b, True, True)
    c = gemm(a, b, trans_a=True, trans_b=True, out_dtype=torch.float32)
    torch.testing.assert_close(c, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)
    old = torch.randn(M, N, device=DEV)
    c = gemm(a, b, trans_a=True, trans_b=True, out=old.clone(), accumulate=True, alpha=0.5)
    torch.testing.assert_close(c, 0.5 * ref + old, rtol=1e-4, atol=1e-3 * K ** 0.5)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(512, 512, 4096), (520, 264, 2048), (1024, 1024, 16384)])
def test_gemm_bf16_ph8_split_k(ta, tb, shape):
    """Few output tiles and a long K (the weight gradient of a <= 2048-wide layer): the
    8-phase kernel's split-K plan -- K-slices into a workspace, one reduction pass with
    the epilogue (accumulate, alpha, bias) -- against the fp32 reference."""
    from distributed_training_pytorch_amd import _native as nat
    M, N, K = shape
    a, b = _ops(M, N, K, ta, tb, torch.bfloat16, 17)
    ref = _ref(a, b, ta, tb)
    args = nat.GemmArgs()
    args.A, args.B, args.M, args.N, args.K = a.data_ptr(), b.data_ptr(), M, N, K
    args.lda, args.ldb = a.stride(0), b.stride(0)
    args.dtype, args.out_dtype, args.trans_a, args.trans_b = nat.DT_BF16, nat.DT_F32, int(ta), int(tb)
    assert nat.load().dtp_gemm_workspace(args) > 0  # the plan applies to these shapes
    old = torch.randn(M, N, device=DEV)
    bias = torch.randn(N, device=DEV)
    c = gemm(a, b, trans_a=ta, trans_b=tb, out=old.clone(), accumulate=True, alpha=0.5, bias=bias)
    torch.testing.assert_close(c, old + 0.5 * ref + bias, rtol=1e-4, atol=2e-3 * K ** 0.5)
    c2 = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32)
    torch.testing.assert_close(c2, ref, rtol=1e-4, atol=2e-3 * K ** 0.5)


def test_compute_shadow_training_is_bit_identical():
    """bf16-compute wide ModelBank: Adam writing the bf16 weight copy in its own pass
    (ComputeShadow) trains bit-identically to casting the fp32 masters before every
    forward, and the shadow equals w.to(bf16) after each step."""
    from distributed_training_pytorch_amd.models.bank import ModelBank
    from distributed_training_pytorch_amd.ops.optim import FlatOptimizer, OptimConfig

    def run(shadow):
        torch.manual_seed(0)
        bank = ModelBank(2, hidden=256, depth=2, compute_dtype=torch.bfloat16).to(DEV)
        sh = bank.compute_shadow() if shadow else None
        opt = FlatOptimizer(bank.flat, bank.flat_grad, OptimConfig(lr=1e-3), shadow=sh)
        g = torch.Generator().manual_seed(1)
        for _ in range(4):
            x = torch.randn(512, 2, generator=g).to(DEV)
            y = torch.randn(512, 1, generator=g).to(DEV)
            bank.zero_grad()
            sum(torch.nn.functional.mse_loss(o, y) for o in bank(x)).backward()
            opt.step()
            if sh is not None:
                assert torch.equal(sh.buf[:, :bank.flat.shape[1]], bank.flat.to(torch.bfloat16))
                assert all(w.data_ptr() % 512 == 0 for w in (m.layers[2].weight._dtp_shadow[1] for m in bank.models))
        return bank.flat.clone(), sh

    a, _ = run(False)
    b, sh = run(True)
    assert sh._token == sh._current()
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(4104, 4360, 256), (8192, 4096, 128)])  # 17 x 18 tiles (ragged); 512 (XCD remap)
def test_gemm_persistent_walk_many_tiles_per_workgroup(ta, tb, shape):
    """The persistent 8-phase kernel with several tiles per workgroup (the next tile's
    operand fill under this tile's epilogue), ragged edges and a tile count that is not a
    multiple of 8, or 2 tiles per workgroup through the XCD remap: the same result as the one-tile-per-workgroup balanced kernel, bit for
    bit (the same K order per output)."""
    torch.manual_seed(11)
    M, N, K = shape
    a = torch.randn(*((K, M) if ta else (M, K)), device="cuda").bfloat16()
    b = torch.randn(*((K, N) if tb else (N, K)), device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    ref = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32, splitk=1, bias=bias, fast=34)
    got = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.float32, splitk=1, bias=bias, fast=37)
    assert torch.equal(ref, got)
    refb = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, act=True, slope=0.1, fast=34)
    gotb = gemm(a, b, trans_a=ta, trans_b=tb, out_dtype=torch.bfloat16, act=True, slope=0.1, fast=37)
    assert torch.equal(refb, gotb)
