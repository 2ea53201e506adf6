"""Numerics of the HIP kernels against plain PyTorch fp32 references of the same op (MI355X)."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    from jumbo_mae_tpu_amd.ops import _ext
    return _ext.load(True)


@pytest.fixture(autouse=True)
def _reset_gemm_variant(request):
    yield
    if "ext" in request.fixturenames:
        request.getfixturevalue("ext").gemm_test_force(0)


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("D", [32, 384, 512, 768, 1024, 2304, 3072])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_layernorm(ext, D, out_dtype):
    torch.manual_seed(0)
    full = torch.randn(5, 9, D, device="cuda") * 3 + 1
    x = full[:, 2:]  # strided [5,7,D] view: 35 rows (D <= 512 runs two rows per wave: an odd tail)
    g = torch.randn(D, device="cuda")
    b = torch.randn(D, device="cuda")
    y, mean, rstd = ext.layernorm_fwd(x, g, b, 1e-6, out_dtype)
    xr = x.detach().clone().double().requires_grad_()
    gr = g.double().requires_grad_()
    br = b.double().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-6).reshape(-1, D)
    tol = 1e-2 if out_dtype == torch.bfloat16 else 1e-5
    assert rel(y, yr) < tol
    dy = torch.randn_like(y)
    dg = torch.zeros(D, device="cuda")
    db = torch.zeros(D, device="cuda")
    dx = ext.layernorm_bwd(dy, x, mean, rstd, g, dg, db, True)[0]
    yr.backward(dy.double())
    assert rel(dx.reshape(-1, D), xr.grad.reshape(-1, D)) < 1e-4
    assert rel(dg, gr.grad) < 1e-4
    assert rel(db, br.grad) < 1e-4


def test_gelu(ext):
    torch.manual_seed(0)
    h = (torch.randn(300, 1024, device="cuda") * 2).bfloat16()
    a = ext.gelu_fwd(h)
    ar = torch.nn.functional.gelu(h.float(), approximate="tanh")
    assert rel(a, ar) < 5e-3
    da = torch.randn_like(h)
    bg = torch.zeros(1024, device="cuda")
    dh = ext.gelu_bwd(h, da, bg)
    hr = h.float().requires_grad_()
    torch.nn.functional.gelu(hr, approximate="tanh").backward(da.float())
    assert rel(dh, hr.grad) < 5e-3
    assert rel(bg, hr.grad.sum(0)) < 5e-3


@pytest.mark.parametrize("M,N", [(1000, 32), (1000, 512), (1000, 768), (1000, 2304), (1000, 4096), (512, 12288)])
def test_colsum(ext, M, N):
    x = torch.randn(M, N, device="cuda").bfloat16()
    acc = torch.ones(N, device="cuda")
    ext.colsum(x, acc)
    assert rel(acc, x.float().sum(0) + 1) < 1e-5


@pytest.mark.parametrize("with_scale", [False, True])
@pytest.mark.parametrize("with_mask", [False, True])
@pytest.mark.parametrize("B,T,D", [(4, 9, 768), (512, 1, 3072), (512, 3, 1024)])  # + jumbo / CLS-row shapes
def test_residual(ext, with_scale, with_mask, B, T, D):
    torch.manual_seed(0)
    full = torch.randn(B, T + 3, D, device="cuda")
    x = full[:, 3:]
    y = torch.randn(B * T, D, device="cuda").bfloat16()
    s = torch.randn(D, device="cuda") if with_scale else None
    m = torch.where(torch.arange(B, device="cuda") % 3 == 0, 0.0, 1.25) if with_mask else None
    out = ext.residual_fwd(x, y, s, m)
    r = y.float().view(B, T, D)
    if s is not None:
        r = r * s
    if m is not None:
        r = r * m.view(B, 1, 1)
    assert rel(out, x + r) < 1e-6
    dout = torch.randn(B, T, D, device="cuda")
    ds = torch.zeros(D, device="cuda") if with_scale else None
    dy = ext.residual_bwd(dout, y if with_scale else None, s, m, ds, torch.bfloat16)
    d = dout * (m.view(B, 1, 1) if m is not None else 1.0)
    if s is not None:
        assert rel(ds, (d * y.float().view(B, T, D)).sum((0, 1))) < 1e-5
        d = d * s
    assert rel(dy, d.reshape(B * T, D)) < 5e-3


def _attn_ref(qkv, H):
    B, S, D3 = qkv.shape
    D = D3 // 3
    hd = D // H
    q, k, v = qkv.double().view(B, S, 3, H, hd).unbind(2)
    z = torch.einsum("bqhd,bkhd->bhqk", q / math.sqrt(hd), k)
    lse = torch.logsumexp(z, -1)
    o = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(z, -1), v).reshape(B, S, D)
    return o, lse


# every kernel the shape dispatch reaches: forward multi-pair (S <= 64) / one-pair, padded and
# exactly-filled key tiles; backward bwd3 4-wave (hd 32), bwd3 8-wave (hd 64, S > 64) and bwd2
# with partial and full 8-element batch groups (hd 64, S <= 64); the 4-wave bwd3's shared last
# key tile (one active tile in the last slot: S 193-208 at SP 224 -- the decoder's 197 -- and 65-80
# at SP 128) with padded and exactly-filled keys, and the plain slot beside it (S 209)
@pytest.mark.parametrize("B,S,H,hd", [(3, 52, 16, 64), (9, 52, 4, 64), (16, 64, 2, 64), (2, 199, 16, 32),
                                      (2, 17, 4, 32), (5, 64, 3, 32), (2, 100, 3, 64), (2, 199, 4, 64),
                                      (3, 224, 2, 64), (2, 128, 2, 32), (1, 33, 5, 64), (32, 19, 4, 64),
                                      (11, 30, 2, 64), (2, 197, 16, 32), (2, 208, 2, 32), (2, 209, 2, 32),
                                      (3, 72, 2, 32)])
def test_attention(ext, B, S, H, hd):
    torch.manual_seed(0)
    D = H * hd
    qkv = (torch.randn(B, S, 3 * D, device="cuda") * 1.5).bfloat16()
    o, lse = ext.attn_fwd(qkv, H)
    orf, lser = _attn_ref(qkv, H)
    assert rel(o, orf) < 1e-2
    assert (lse.double() - lser).abs().max().item() < 2e-2
    do = torch.randn(B, S, D, device="cuda").bfloat16()
    dqkv = ext.attn_bwd(do, qkv, o, lse, H)
    dbias = torch.full((3 * D,), 0.5, device="cuda")
    dqkv2 = ext.attn_bwd(do, qkv, o, lse, H, dbias)  # fused QKV-bias colsum (accumulates)
    assert torch.equal(dqkv, dqkv2)
    ref_b = dqkv.double().sum((0, 1)) + 0.5
    assert (dbias.double() - ref_b).abs().max().item() < 2e-2 * ref_b.abs().max().item() + 1e-2
    qr = qkv.double().requires_grad_()
    o2, _ = _attn_ref(qr, H)
    o2.backward(do.double())
    g = qr.grad.view(B, S, 3, D)
    d = dqkv.view(B, S, 3, D)
    for i in range(3):
        assert rel(d[:, :, i], g[:, :, i]) < 2e-2, i
    for _ in range(3):  # one writer per element, fixed-order sums (no float atomics): bit-identical reruns
        db2 = torch.full((3 * D,), 0.5, device="cuda")
        assert torch.equal(ext.attn_bwd(do, qkv, o, lse, H, db2), dqkv) and torch.equal(db2, dbias)


@pytest.mark.parametrize("B,S,H,hd", [(3, 52, 4, 64), (2, 199, 4, 32), (2, 199, 3, 64), (5, 17, 2, 32),
                                      (9, 30, 2, 64), (2, 100, 2, 32), (3, 72, 2, 32)])
def test_attention_dropout(ext, B, S, H, hd):
    """Dropout on the attention probabilities inside the fused kernels (forward: masked P.V with
    the undropped row statistics; backward: the mask regenerated from the seed) against an fp64
    reference with the mirrored mask (ops/dropout.py keep_mask_rows)."""
    from jumbo_mae_tpu_amd.ops import dropout as Dr
    torch.manual_seed(0)
    rate = 0.2
    D = H * hd
    qkv = (torch.randn(B, S, 3 * D, device="cuda") * 1.5).bfloat16()
    seed = torch.tensor([0x5EED_1234_5678], dtype=torch.int64, device="cuda")
    o, lse = ext.attn_fwd(qkv, H, seed, rate)
    m = Dr.keep_mask_rows(seed.cpu(), B * H * S, S, rate).view(B, H, S, S).cuda().double() / (1 - rate)
    qr = qkv.double().requires_grad_()
    q, k, v = qr.view(B, S, 3, H, hd).unbind(2)
    z = torch.einsum("bqhd,bkhd->bhqk", q / math.sqrt(hd), k)
    lser = torch.logsumexp(z, -1)
    orf = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(z, -1) * m, v).reshape(B, S, D)
    assert rel(o, orf) < 1e-2
    assert (lse.double() - lser).abs().max().item() < 2e-2
    do = torch.randn(B, S, D, device="cuda").bfloat16()
    dbias = torch.zeros(3 * D, device="cuda")
    dqkv = ext.attn_bwd(do, qkv, o, lse, H, dbias, seed, rate)
    orf.backward(do.double())
    g = qr.grad.view(B, S, 3, D)
    d = dqkv.view(B, S, 3, D)
    for i in range(3):
        assert rel(d[:, :, i], g[:, :, i]) < 2e-2, i
    assert rel(dbias, qr.grad.sum((0, 1))) < 2e-2
    o0, _ = ext.attn_fwd(qkv, H)
    assert rel(o0, orf) > 0.05  # the mask is live


@pytest.mark.parametrize("S,n", [(4, 4096), (512, 3072), (37, 1024)])
def test_splitk_reduce_add(ext, S, n):
    part = torch.randn(S, n, device="cuda")
    g = torch.randn(n, device="cuda")
    ref = g.double() + part.double().sum(0)
    ext.splitk_reduce_add(part, g)
    assert (g.double() - ref).abs().max().item() < 1e-4


def test_patchify(ext):
    from jumbo_mae_tpu_amd.ops.mae import normalize_images
    from jumbo_mae_tpu_amd.utils.mae import extract_patches_nchw
    img = torch.randint(0, 256, (3, 3, 224, 224), dtype=torch.uint8, device="cuda")
    out = ext.patchify_normalize(img, 16)
    ref = extract_patches_nchw(normalize_images(img), 16)
    assert (out - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("kind", ["adamw", "lamb", "lars", "sgd"])
@pytest.mark.parametrize("clip", [0.0, 0.5])
def test_optimizer_hip_matches_torch(kind, clip):
    from jumbo_mae_tpu_amd.config import ViTConfig, DecoderConfig
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    vc = ViTConfig(layers=2, dim=64, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d")
    dc = DecoderConfig(dec_layers=1, dec_dim=32, dec_heads=2, image_size=32, patch_size=8)
    sched = warmup_cosine_decay_schedule(1e-6, 1e-2, 3, 10, 1e-5)
    res = []
    init = None
    for dev, dt in (("cuda", torch.bfloat16), ("cpu", torch.float32)):
        m = PretrainModel(vc, dc).to(dev, dt, seed=0)
        if init is None:
            init = m.store.master.cpu().clone()
        m.store.master.copy_(init)
        m.store.sync_shadow()
        opt = FlatOptimizer(m.store, kind, sched, b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.05,
                            lr_decay=0.75, num_layers=2, clip_grad=clip)
        gen = torch.Generator().manual_seed(1)
        for _ in range(3):
            m.store.grad.copy_(torch.randn(m.store.total, generator=gen).to(dev))
            opt.step()
        res.append(m.store.master.cpu())
        if dev == "cuda":
            assert torch.allclose(m.store.shadow.float().cpu(), m.store.master.cpu(), rtol=1e-2, atol=1e-3)
    assert rel(res[0], res[1]) < 1e-5


@pytest.mark.parametrize("path", [0, 1, 2])
@pytest.mark.parametrize("M,N,K,gelu", [(512, 256, 64, False), (300, 196, 128, True), (1000, 1536, 512, False),
                                        (257, 260, 192, True), (16100, 2048, 128, True), (40000, 520, 64, False)])
def test_gemm_nt(ext, M, N, K, gelu, path):
    """Hand-written MFMA GEMMs (csrc/gemm.hip) vs an fp32 reference, ragged M / N included: by shape
    (path 0: the 128 x 192 narrow kernel below M = 4096, the 256 x 256 kernels otherwise), the
    64-deep main loop everywhere (path 1; by shape it runs only at K % 128 == 64) and the 4-phase
    kernels at every M (path 2)."""
    ext.gemm_test_force(path)
    torch.manual_seed(0)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.1).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    outs = ext.gemm_nt(x, w, b, gelu)
    ref = x.float() @ w.float().t() + b
    assert rel(outs[0], ref) < 1e-2
    if gelu:
        g_ref = torch.nn.functional.gelu(outs[0].float(), approximate="tanh")
        assert rel(outs[1], g_ref) < 1e-2


@pytest.mark.parametrize("rows", [224, 192, 160, 256])
@pytest.mark.parametrize("M,N,K,lda", [(5000, 776, 256, 256), (4500, 260, 128, 192), (6272, 1024, 512, 512),
                                       (4097, 512, 384, 448)])
def test_gemm_nt_short_rows(ext, M, N, K, lda, rows):
    """4-phase kernel at forced tile heights (224 / 192 rows: p4_mainloop MTL = 3 / 2) against fp32,
    every epilogue (bias, GELU pair, gelu' / gelu, GELU only, dGELU and dGELU-multiply with the
    column-partial bias gradient), ragged M, N % 8 != 0 (register epilogue) and strided A rows."""
    ext.gemm_test_force(2, rows)
    torch.manual_seed(0)
    xa = (torch.rand(M, lda, device="cuda") * 2 - 1).bfloat16()
    x = xa[:, :K]
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.1).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    ref = x.float() @ w.float().t() + b
    out = ext.gemm_nt(x, w, b)[0]
    assert rel(out, ref) < 1e-2
    h, g = ext.gemm_nt(x, w, b, True)
    assert rel(h, ref) < 1e-2
    assert rel(g, torch.nn.functional.gelu(h.float(), approximate="tanh")) < 1e-2
    (go,) = ext.gemm_nt(x, w, b, True, True)
    assert rel(go, g) < 1e-2
    if N % 8:
        return
    dq, g2 = ext.gemm_nt(x, w, b, True, False, True)
    hr = h.float()
    t = torch.tanh(0.7978845608028654 * (hr + 0.044715 * hr ** 3))
    dref = 0.5 * (1 + t) + 0.5 * hr * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * hr * hr)
    d = _gd_check(dq, dref)
    assert rel(g2, g) < 1e-2
    # data gradient through the GELU: [M, K'] x [N, K']^T * gelu'(pre)
    dy = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    dg = (dy.float() @ w.float().t()).bfloat16().float()
    for deriv, aux, fac in ((False, h, dref), (True, dq, d)):
        db = torch.full((N,), 0.25, device="cuda")
        o = ext.gemm_nt_dgelu(dy, w, aux, db, deriv)
        r = dg * fac
        assert rel(o, r) < 1e-2, deriv
        assert rel(db - 0.25, r.sum(0)) < 1e-2, deriv


def _gd_check(dq, dref):
    """uint8 gelu' codes of the fused FF1 forward (csrc/common.h gd_code) against the fp32 derivative
    of the same bf16 pre-activation: the torch mirror's code up to one step (fma vs two roundings at
    exact ties), the decoded value within half a step.  Returns the decoded fp32 gelu'."""
    from jumbo_mae_tpu_amd.ops import prims as P
    assert dq.dtype == torch.uint8 and dq.shape == dref.shape
    assert (dq.int() - P.gd_encode(dref).int()).abs().max().item() <= 1
    d = P.gd_decode(dq, dtype=torch.float32)
    assert (d - dref).abs().max().item() <= 0.5 / P.GD_Q + 1e-4
    return d


def test_gemm_tile_rows_choice(ext):
    """Automatic tile height: the FF1 forward / FF2 data gradient of ViT-L pretraining (M = 25088,
    N = 4096: 6.1 waves of 256-row tiles) takes 224-row tiles (exactly 7 waves) on 256 CUs; the
    QKV forward (N = 3072, 4.9 waves) stays at 256."""
    if torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("wave-fill expectations assume 256 CUs")
    assert ext.gemm_nt_tiles(25088, 4096, 1024, 6, 1024) == 112 * 16
    assert ext.gemm_nt_tiles(26624, 3072, 1024, 0, 1024) == 104 * 12


@pytest.mark.parametrize("B,S,H,hd", [(2, 300, 4, 64), (1, 787, 3, 64), (2, 225, 2, 32), (1, 787, 2, 32)])
def test_attention_long_sequence_path(ext, B, S, H, hd):
    """S > attn_max_seq() (finetune at 448 px: S = 787) runs the tile-streamed online-softmax
    kernels (attn_fwd_long / attn_bwd_dq / attn_bwd_dkv); fp64 reference incl. gradients, through
    the prims (the QKV bias gradient is then left to the caller)."""
    from jumbo_mae_tpu_amd.ops import prims as P
    assert S > ext.attn_max_seq()
    torch.manual_seed(0)
    qkv = (torch.randn(B, S, 3 * H * hd, device="cuda") * 1.5).bfloat16()
    o, lse = P.attn_fwd(qkv, H)
    orf, lser = _attn_ref(qkv, H)
    assert rel(o, orf) < 1e-2
    assert (lse.double() - lser).abs().max().item() < 2e-2
    do = torch.randn(B, S, H * hd, device="cuda").bfloat16()
    dqkv, done = P.attn_bwd(do, qkv, o, lse, H)
    assert not done
    qr = qkv.double().requires_grad_()
    o2, _ = _attn_ref(qr, H)
    o2.backward(do.double())
    g = qr.grad.view(B, S, 3, H * hd)
    d = dqkv.view(B, S, 3, H * hd)
    for i in range(3):
        assert rel(d[:, :, i], g[:, :, i]) < 2e-2, i
    dqkv2, _ = P.attn_bwd(do, qkv, o, lse, H)
    assert torch.equal(dqkv, dqkv2)  # one writer per element: deterministic


@pytest.mark.parametrize("path", [0, 2, 1])
@pytest.mark.parametrize("M,N,K", [(512, 256, 64), (1000, 1536, 512), (300, 512, 128), (5000, 776, 256)])
def test_gemm_nt_dgelu(ext, M, N, K, path):
    """FF2 data gradient through the GELU with the FF1 bias gradient (csrc/gemm.hip EPI_DGELU)."""
    ext.gemm_test_force(path)
    torch.manual_seed(0)
    dy = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w2t = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.1).bfloat16()
    pre = (torch.randn(M, N, device="cuda") * 2).bfloat16()
    db = torch.full((N,), 0.25, device="cuda")
    out = ext.gemm_nt_dgelu(dy, w2t, pre, db)
    dg = (dy.float() @ w2t.float().t()).bfloat16().float()
    x = pre.float()
    t = torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3))
    d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * x * x)
    ref = dg * d
    assert rel(out, ref) < 1e-2
    assert rel(db - 0.25, ref.sum(0)) < 1e-2


@pytest.mark.parametrize("R,C", [(1024, 3072), (512, 2048), (72, 136)])
def test_transpose_bf16(ext, R, C):
    x = torch.randn(R, C, device="cuda").bfloat16()
    y = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    ext.transpose_bf16(x, y)
    assert torch.equal(y, x.t())


@pytest.mark.parametrize("M,N,K", [(4096, 256, 512), (3000, 512, 256), (512, 768, 1024), (26624, 1024, 256),
                                   (101888, 512, 512), (200, 256, 256), (480, 256, 256), (25088, 1024, 4096)])
def test_gemm_tn_wgrad(ext, M, N, K):
    """Weight-gradient TN MFMA GEMM (csrc/gemm_tn.hip): G += dy^T x, split over M (fp32 slices +
    reduce), ragged M, run twice (accumulation); plain and segmented (the 4-phase kernel at 64-row
    segments, the 32-row-step kernel otherwise)."""
    torch.manual_seed(0)
    dy = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16()
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    g = torch.randn(N, K, device="cuda")
    ref = g.double() + dy.double().t() @ x.double()
    S = ext.gemm_tn_wgrad(dy, x, g)
    assert S >= 1 and (S > 1 or M < 8192)
    assert rel(g, ref) < 1e-4
    g3 = torch.zeros_like(g)
    ext.gemm_tn_wgrad(dy, x, g3)
    ext.gemm_tn_wgrad(dy, x, g3)
    assert rel(g3, 2 * (dy.double().t() @ x.double())) < 1e-4
    for n in (4, 5):
        if M % n or (M // n) % 32:
            continue
        rows = M // n
        g2 = ref.float().clone()
        ref2 = ref + dy.double().t() @ x.double()
        ext.gemm_tn_wgrad_seg([dy[i * rows:(i + 1) * rows] for i in range(n)],
                              [x[i * rows:(i + 1) * rows] for i in range(n)], g2)
        assert rel(g2, ref2) < 1e-4, n


@pytest.mark.parametrize("M,shapes", [(4096, [(256, 1024), (1024, 256)]), (26624, [(1024, 1024), (3072, 1024)]),
                                      (5000, [(512, 256), (256, 512), (768, 256)]), (25088, [(1024, 4096), (4096, 1024)])])
def test_gemm_tn_wgrad_group(ext, M, shapes):
    """Grouped TN weight gradients (one grid over several problems with the same M, ragged M
    included) == separate fp64 references, accumulated into existing gradients; run twice."""
    torch.manual_seed(0)
    dys = [(torch.rand(M, n, device="cuda") * 2 - 1).bfloat16() for n, _ in shapes]
    xs = [(torch.rand(M, k, device="cuda") * 2 - 1).bfloat16() for _, k in shapes]
    gs = [torch.randn(n, k, device="cuda") for n, k in shapes]
    refs = [g.double() + 2 * (d.double().t() @ x.double()) for g, d, x in zip(gs, dys, xs)]
    S = ext.gemm_tn_wgrad_group(dys, xs, gs)
    assert S >= 1
    ext.gemm_tn_wgrad_group(dys, xs, gs)
    for g, r in zip(gs, refs):
        assert rel(g, r) < 1e-4


@pytest.mark.parametrize("M,N,K", [(4096, 256, 512), (26624, 1024, 256), (8192, 2048, 512)])
def test_gemm_tn_wgrad_store(ext, M, N, K):
    """Store mode of the TN weight gradient (first contribution of a step): G's previous contents
    are ignored -- split-K reduce without reading G, one-split launches writing G -- plain, grouped
    (mixed store flags) and segmented."""
    torch.manual_seed(0)
    dy = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16()
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    ref = dy.double().t() @ x.double()
    g = torch.full((N, K), 1e4, device="cuda")
    ext.gemm_tn_wgrad(dy, x, g, True)
    assert rel(g, ref) < 1e-4
    ext.gemm_tn_wgrad(dy, x, g)  # accumulate on top
    assert rel(g, 2 * ref) < 1e-4
    g1, g2 = torch.full((N, K), 1e4, device="cuda"), torch.ones(K, N, device="cuda")
    ext.gemm_tn_wgrad_group([dy, x], [x, dy], [g1, g2], [True, False])
    assert rel(g1, ref) < 1e-4 and rel(g2, 1 + ref.t()) < 1e-4
    rows = M // 4
    g3 = torch.full((N, K), -3.0, device="cuda")
    ext.gemm_tn_wgrad_seg([dy[i * rows:(i + 1) * rows] for i in range(4)],
                          [x[i * rows:(i + 1) * rows] for i in range(4)], g3, True)
    assert rel(g3, ref) < 1e-4


def test_zero_ranges(ext):
    """Multi-range zeroing of a flat buffer (ParamStore.zero_grad): only the listed ranges change."""
    buf = torch.arange(100000, device="cuda", dtype=torch.float32) + 1
    ranges = [(0, 5), (17, 4096), (9000, 1), (20000, 50000), (99990, 10)]
    desc = torch.tensor(ranges, dtype=torch.int64, device="cuda")
    blocks = sum(-(-c // 4096) for _, c in ranges)
    ext.zero_ranges(buf, desc, blocks)
    ref = torch.arange(100000, device="cuda", dtype=torch.float32) + 1
    for a, c in ranges:
        ref[a:a + c] = 0
    assert torch.equal(buf, ref)


@pytest.mark.parametrize("nb,rows", [(24, 512), (5, 128), (3, 64)])
def test_gemm_tn_wgrad_seg_group(ext, nb, rows):
    """Grouped + segmented TN weight gradients (the jumbo MLP's W1 / W2 over the per-layer row
    blocks, read in place) == fp64 references, accumulated into existing gradients."""
    torch.manual_seed(0)
    shapes = [(1024, 256), (256, 1024)]
    dys = [[(torch.rand(rows, n, device="cuda") * 2 - 1).bfloat16() for _ in range(nb)] for n, _ in shapes]
    xs = [[(torch.rand(rows, k, device="cuda") * 2 - 1).bfloat16() for _ in range(nb)] for _, k in shapes]
    gs = [torch.randn(n, k, device="cuda") for n, k in shapes]
    refs = [g.double() + torch.cat(d).double().t() @ torch.cat(x).double() for g, d, x in zip(gs, dys, xs)]
    ext.gemm_tn_wgrad_seg_group(dys, xs, gs)
    for g, r in zip(gs, refs):
        assert rel(g, r) < 1e-4


@pytest.mark.parametrize("T0", [0, 3])
@pytest.mark.parametrize("with_scale", [False, True])
def test_residual_ln_fwd(ext, T0, with_scale):
    """Fused residual + LayerNorm == residual_fwd followed by layernorm_fwd (bit-identical math)."""
    torch.manual_seed(0)
    B, T, D = 5, 52, 1024
    x = torch.randn(B, T, D, device="cuda")
    y = torch.randn(B * T, D, device="cuda").bfloat16()
    s = torch.rand(D, device="cuda") if with_scale else None
    mask = (torch.rand(B, device="cuda") > 0.3).float() / 0.7
    g, b = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda")
    x1, h, mu, rs = ext.residual_ln_fwd(x, y, s, mask, g, b, 1e-6, T0)
    x1r = ext.residual_fwd(x, y, s, mask)
    hr, mur, rsr = ext.layernorm_fwd(x1r[:, T0:], g, b, 1e-6, torch.bfloat16)
    assert torch.equal(x1, x1r)
    assert (h.float() - hr.float()).abs().max().item() <= 0.0625
    assert torch.allclose(mu, mur, atol=1e-6) and torch.allclose(rs, rsr, rtol=1e-5)


@pytest.mark.parametrize("D", [512, 1024])
def test_residual_ln_fwd_partial_rows(ext, D):
    """R0 = 3 (the jumbo block's hand-off): rows t >= 3 get the residual into ``out``, rows t < 3 of
    ``out`` are already final; the LayerNorm covers all rows == residual_fwd on the patch rows then
    layernorm_fwd over the assembled tensor."""
    torch.manual_seed(0)
    B, T, C = 5, 52, 3
    x = torch.randn(B, T, D, device="cuda")
    y = torch.randn(B * (T - C), D, device="cuda").bfloat16()
    s = torch.rand(D, device="cuda")
    mask = (torch.rand(B, device="cuda") > 0.3).float() / 0.7
    g, b = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda")
    out = torch.empty(B, T, D, device="cuda")
    out[:, :C] = torch.randn(B, C, D, device="cuda")
    cls = out[:, :C].clone()
    x1, h, mu, rs = ext.residual_ln_fwd(x, y, s, mask, g, b, 1e-6, 0, C, out)
    assert x1.data_ptr() == out.data_ptr() and torch.equal(out[:, :C], cls)
    ref = torch.empty_like(out)
    ref[:, :C] = cls
    ref[:, C:] = ext.residual_fwd(x[:, C:], y, s, mask)
    assert torch.equal(out, ref)
    hr, mur, rsr = ext.layernorm_fwd(ref, g, b, 1e-6, torch.bfloat16)
    assert (h.float() - hr.float()).abs().max().item() <= 0.0625
    assert torch.allclose(mu, mur, atol=1e-6) and torch.allclose(rs, rsr, rtol=1e-5)


@pytest.mark.parametrize("path", [0, 2, 1])
@pytest.mark.parametrize("M,N,K,S", [(512, 3072, 12288, 10), (300, 512, 4096, 3), (512, 256, 1024, 16),
                                     (128, 2304, 9216, 16), (128, 1000, 2304, 4)])
def test_gemm_nt_splitk(ext, M, N, K, S, path):
    """Split-K MFMA GEMM (fp32 partial tiles + bf16 reduce with bias), ragged M."""
    ext.gemm_test_force(path)
    torch.manual_seed(0)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    out = ext.gemm_nt_splitk(x, w, b, S)
    ref = x.float() @ w.float().t() + b
    assert rel(out, ref) < 1e-2


@pytest.mark.parametrize("T0,view_y,with_scale", [(0, False, True), (3, False, True), (0, True, True),
                                                  (3, True, False)])
@pytest.mark.parametrize("B,T,D", [(6, 52, 1024), (5, 51, 512)])
def test_layernorm_bwd_fused_residual(ext, T0, view_y, with_scale, B, T, D):
    """LN backward with the consumer's residual backward fused in == layernorm_bwd followed by
    residual_bwd on the rows t >= T0 (y as a contiguous slab or a strided view into a buffer);
    D = 512 with an odd row count: the two-rows-per-wave decoder variant and its tail."""
    torch.manual_seed(0)
    x = torch.randn(B, T, D, device="cuda") * 2
    g, bt = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda")
    _, mean, rstd = ext.layernorm_fwd(x, g, bt, 1e-6, torch.bfloat16)
    dy = torch.randn(B * T, D, device="cuda").bfloat16()
    dres = torch.randn(B, T, D, device="cuda")
    Tr = T - T0
    s = torch.rand(D, device="cuda") if with_scale else None
    mask = (torch.rand(B, device="cuda") > 0.3).float() / 0.7
    if view_y:
        ybuf = torch.randn(B, T + 2, D, device="cuda").bfloat16()
        y = ybuf[:, 2:2 + Tr]
        obuf = torch.zeros_like(ybuf)
        out = obuf[:, 2:2 + Tr]
    else:
        y = torch.randn(B * Tr, D, device="cuda").bfloat16()
        out = None
    z = lambda: torch.zeros(D, device="cuda")  # noqa: E731
    dg1, db1, ds1, dbi1 = z(), z(), z(), z()
    dx1, dyr = ext.layernorm_bwd(dy, x, mean, rstd, g, dg1, db1, True, dres, None, y, s, mask,
                                 ds1 if with_scale else None, dbi1, T0, out)
    dg2, db2, ds2, dbi2 = z(), z(), z(), z()
    dx2 = ext.layernorm_bwd(dy, x, mean, rstd, g, dg2, db2, True, dres)[0]
    # the two instantiations may contract the dx expression into FMAs differently: fp32 rounding
    assert torch.allclose(dx1, dx2, rtol=1e-5, atol=1e-6)
    assert rel(dg1, dg2) < 1e-5 and rel(db1, db2) < 1e-5
    if view_y:
        o2 = torch.zeros_like(ybuf)
        ref = ext.residual_bwd(dx2[:, T0:], y, s, mask, ds2 if with_scale else None, torch.bfloat16, dbi2,
                               o2[:, 2:2 + Tr])
        outside = torch.ones_like(obuf, dtype=torch.bool)
        outside[:, 2:2 + Tr] = False
        assert (obuf[outside] == 0).all() and (o2[outside] == 0).all()  # nothing outside the view touched
        assert rel(obuf, o2) < 1e-3  # bf16: a few 1-ulp rounding flips
    else:
        ref = ext.residual_bwd(dx2[:, T0:], y, s, mask, ds2 if with_scale else None, torch.bfloat16, dbi2)
    assert rel(dyr, ref) < 1e-3
    if with_scale:
        assert rel(ds1, ds2) < 1e-5
    assert rel(dbi1, dbi2) < 1e-4  # colsums of bf16 values: rounding flips


@pytest.mark.parametrize("gamma_kind", ["init", "trained", "zeros_tiny"])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("B,T,D", [(6, 52, 1024), (5, 51, 512), (4, 49, 768)])
def test_layernorm_bwd_from_h(ext, gamma_kind, fused, B, T, D):
    """LN backward that rebuilds x-hat from the forward's bf16 output h (hx / beta) against the
    fp64 LayerNorm autograd: gamma = 1, beta = 0 (init: the h path); trained-like gamma / beta with
    |beta| > |gamma| in a third of the columns, and gamma with exact zeros and 1e-6 entries (the
    launch falls back to reading x).  Same tolerance class as the x path: dx / dgamma / dbeta within 1e-2 relative
    (bf16-level x-hat), and the x-path result within 1e-2 of it."""
    torch.manual_seed(0)
    x = torch.randn(B, T, D, device="cuda") * 2 + 0.5
    if gamma_kind == "init":
        g, bt = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
    elif gamma_kind == "trained":
        g = torch.randn(D, device="cuda") * 0.5 + 1.0
        bt = torch.randn(D, device="cuda") * 0.5
        bt[::3] = 2.0 * g[::3].abs() + 0.1  # |beta| > |gamma|: x path for those chunks
    else:
        g = torch.rand(D, device="cuda") + 0.5
        g[5] = 0.0
        g[100:104] = 1e-6
        g[-1] = -1e-6
        bt = torch.randn(D, device="cuda") * 0.1
    h, mean, rstd = ext.layernorm_fwd(x, g, bt, 1e-6, torch.bfloat16)
    dy = torch.randn(B * T, D, device="cuda").bfloat16()
    dres = torch.randn(B, T, D, device="cuda")
    z = lambda: torch.zeros(D, device="cuda")  # noqa: E731
    if fused:
        y = torch.randn(B * T, D, device="cuda").bfloat16()
        mask = torch.ones(B, device="cuda")
        dg1, db1, dbi1 = z(), z(), z()
        dx1, dyr1 = ext.layernorm_bwd(dy, x, mean, rstd, g, dg1, db1, True, dres, None, y, None, mask, None, dbi1, 0,
                                      None, hx=h, beta=bt)
        dg2, db2, dbi2 = z(), z(), z()
        dx2, dyr2 = ext.layernorm_bwd(dy, x, mean, rstd, g, dg2, db2, True, dres, None, y, None, mask, None, dbi2, 0)
        assert rel(dyr1, dyr2) < 1e-2 and rel(dbi1, dbi2) < 1e-2
    else:
        dg1, db1 = z(), z()
        dx1 = ext.layernorm_bwd(dy, x, mean, rstd, g, dg1, db1, True, dres, hx=h, beta=bt)[0]
        dg2, db2 = z(), z()
        dx2 = ext.layernorm_bwd(dy, x, mean, rstd, g, dg2, db2, True, dres)[0]
    xr = x.double().requires_grad_()
    gr, br = g.double().requires_grad_(), bt.double().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-6)
    yr.backward(dy.double().reshape(B, T, D))
    dxr = xr.grad + dres.double()
    for ours in (dx1, dx2):
        assert rel(ours, dxr) < 1e-2
    assert rel(dg1, gr.grad) < 1e-2 and rel(db1, br.grad) < 1e-5
    assert rel(dx1, dx2) < 1e-2 and rel(dg1, dg2) < 1e-2
    if gamma_kind == "zeros_tiny":  # columns with zero / tiny gamma took the exact path: dgamma there
        cols = [5, 100, 101, 102, 103, D - 1]
        assert torch.allclose(dg1[cols].double(), gr.grad[cols], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("kind", ["store", "gelu", "gelu_only", "dgelu"])
@pytest.mark.parametrize("M,N,K", [(4352, 4096, 1024), (4200, 4096, 512), (25472, 768, 3072)])
def test_gemm_nt_tail_split(ext, kind, M, N, K):
    """Last partial wave of tiles computed split-K + finish kernel == the plain launch (path 2 at
    256-row tiles: no tail split)."""
    torch.manual_seed(5)
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    pre = (torch.randn(M, N, device="cuda") * 2).bfloat16()
    outs = []
    for tail in (0, 1):
        ext.gemm_test_force(0 if tail else 2, 256)
        if kind == "dgelu":
            db = torch.zeros(N, device="cuda")
            outs.append((ext.gemm_nt_dgelu(A, W, pre, db), db))
        else:
            outs.append(tuple(ext.gemm_nt(A, W, b, kind != "store", kind == "gelu_only")))
    ext.gemm_test_force(0)
    ref = A.float() @ W.float().t()
    for o0, o1 in zip(outs[0], outs[1]):
        assert o0.shape == o1.shape
        assert rel(o1, o0) < 5e-3
    if kind == "store":
        assert rel(outs[1][0], ref + b) < 1e-2
    if kind == "dgelu":
        assert rel(outs[1][1], outs[0][1]) < 1e-3


def test_layernorm_fwd_also_bf16(ext):
    """fp32 LN output plus its bf16 copy from the same pass == .bfloat16() of the fp32 output."""
    torch.manual_seed(0)
    full = torch.randn(5, 7, 3072, device="cuda") * 2 + 0.5
    x = full[:, 4:]  # strided [5, 3, 3072] view (the jumbo CLS rows)
    g, b = torch.randn(3072, device="cuda"), torch.randn(3072, device="cuda")
    y, m, r = ext.layernorm_fwd(x, g, b, 1e-6, torch.float32)
    y2, m2, r2, yb = ext.layernorm_fwd(x, g, b, 1e-6, torch.float32, True)
    assert torch.equal(y, y2) and torch.equal(m, m2) and torch.equal(r, r2)
    assert yb.dtype == torch.bfloat16 and torch.equal(yb, y.bfloat16())


def test_gemm_splitk_fused_fp32_add(ext):
    """Split-K NT GEMM returning A.B^T + add in fp32 (add = a strided fp32 view, the jumbo-MLP input
    gradient path) == fp32 reference; bias variant too."""
    torch.manual_seed(0)
    M, N, K = 512, 3072, 12288
    A = (torch.randn(M, K, device="cuda") * 0.05).bfloat16()
    B = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    big = torch.randn(M, 3, N, device="cuda")
    add = big[:, 1]  # [M, N], row stride 3N
    ref = A.float() @ B.float().t()
    out = ext.gemm_nt_splitk(A, B, None, 10, add)
    assert out.dtype == torch.float32 and out.shape == (M, N)
    assert rel(out, ref + add) < 1e-5 + 1e-3 * ref.norm().item() / (ref + add).norm().item()
    bias = torch.randn(N, device="cuda")
    out_b = ext.gemm_nt_splitk(A, B, bias, 10, add)
    assert rel(out_b, ref + bias + add) < 2e-3
    # bf16 path unchanged
    assert rel(ext.gemm_nt_splitk(A, B, None, 10), ref) < 1e-2


def test_linear_dgrad_fp32_add_one_split(ext):
    """Jumbo W1 data gradient at the headline's 2048-row micro-batch: no split-K plan, so the fp32
    addend goes through ONE fp32 split + the reduce's add (ops/prims.py linear_dgrad) == fp32
    reference, on the same narrow kernel as the bf16 path."""
    from jumbo_mae_tpu_amd.ops import prims as P

    torch.manual_seed(0)
    M, N, K = 2048, 3072, 12288
    assert P.splitk_plan(M, N, K) == 0
    A = (torch.randn(M, K, device="cuda") * 0.05).bfloat16()
    B = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    add = torch.randn(M, 3, N, device="cuda")[:, 1]
    ref = A.float() @ B.float().t()
    out = ext.gemm_nt_splitk(A, B, None, 1, add)
    assert out.dtype == torch.float32 and out.shape == (M, N)
    assert rel(out, ref + add) < 1e-5 + 1e-3 * ref.norm().item() / (ref + add).norm().item()


@pytest.mark.parametrize("variant", [12, 24, 84])
@pytest.mark.parametrize("M,N,K", [(1000, 512, 256), (600, 1000, 128)])
def test_gemm_gelu_saved_derivative(ext, M, N, K, variant):
    """FF1 forward saving gelu'(h) (EPI_GELU_D) and the FF2 data gradient multiplying by it
    (EPI_DMUL) == the h-saving pair (EPI_GELU / EPI_DGELU); the unfused gelu_bwd(deriv) too."""
    torch.manual_seed(0)
    x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    h, g = ext.gemm_nt(x, w, b, True)
    gp, g2 = ext.gemm_nt(x, w, b, True, False, True)
    assert torch.equal(g, g2)
    hf = h.float()
    t = torch.tanh(0.7978845608028654 * (hf + 0.044715 * hf ** 3))
    dref = 0.5 * (1 + t) + 0.5 * hf * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * hf * hf)
    _gd_check(gp, dref)
    dy = (torch.randn(M, 384, device="cuda") * 0.5).bfloat16()
    w2t = (torch.randn(N, 384, device="cuda") * 0.05).bfloat16()
    db1, db2 = torch.zeros(N, device="cuda"), torch.zeros(N, device="cuda")
    d1 = ext.gemm_nt_dgelu(dy, w2t, h, db1)
    d2 = ext.gemm_nt_dgelu(dy, w2t, gp, db2, True)
    assert rel(d2, d1) < 1e-2 and rel(db2, db1) < 1e-2
    da = (torch.randn(M, N, device="cuda")).bfloat16()
    bg1, bg2 = torch.zeros(N, device="cuda"), torch.zeros(N, device="cuda")
    e1 = ext.gelu_bwd(h, da, bg1)
    from jumbo_mae_tpu_amd.ops import prims as P
    e2 = ext.gelu_bwd(P.gd_decode(gp), da, bg2, True)
    assert rel(e2, e1) < 1e-2 and rel(bg2, bg1) < 1e-2


@pytest.mark.parametrize("M,N,K", [(4352, 1024, 256), (512, 12288, 192)])
def test_gemm_gelu_saved_derivative_dropout(ext, M, N, K):
    """FF hidden dropout inside the GELU_D epilogue (4-phase and narrow kernels): gelu(h) is masked
    and scaled by 1 / keep, the gelu' codes hold the unscaled derivative where kept and exact 0 where
    dropped, and the DMUL data gradient decoding them with ``rate`` == dg * gelu'(h) * mask / keep."""
    from jumbo_mae_tpu_amd.ops import dropout as Dr
    from jumbo_mae_tpu_amd.ops import prims as P
    torch.manual_seed(3)
    rate = 0.1
    x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    seed = torch.tensor([0x5EED], dtype=torch.int64, device="cuda")
    h, g = ext.gemm_nt(x, w, b, True)
    gp, gd = ext.gemm_nt(x, w, b, True, False, True, seed, rate)
    keep = Dr.keep_mask(seed.cpu(), M * N, rate).view(M, N).cuda()
    scale = 1.0 / (1.0 - rate)
    # kept: bf16 of the fp32 gelu(h) / keep (the kernel rounds once; bf16(g) / keep would round twice)
    assert bool((gd[~keep] == 0).all())
    want = g.float()[keep] * scale
    assert ((gd.float()[keep] - want).abs() <= want.abs() * 2 ** -7 + 1e-30).all()
    hf = h.float()
    t = torch.tanh(0.7978845608028654 * (hf + 0.044715 * hf ** 3))
    dref = 0.5 * (1 + t) + 0.5 * hf * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * hf * hf)
    assert bool((gp[~keep] == P.GD_Z).all())
    _gd_check(torch.where(keep, gp, P.gd_encode(dref)), dref)
    dy = (torch.randn(M, 384, device="cuda") * 0.5).bfloat16()
    w2t = (torch.randn(N, 384, device="cuda") * 0.05).bfloat16()
    db = torch.zeros(N, device="cuda")
    out = ext.gemm_nt_dgelu(dy, w2t, gp, db, True, rate)
    ref = (dy.float() @ w2t.float().t()).bfloat16().float() * P.gd_decode(gp, rate, torch.float32)
    assert rel(out, ref) < 1e-2 and rel(db, ref.sum(0)) < 1e-2
    assert bool((out[~keep] == 0).all())


def test_transpose_bf16_batch(ext):
    """All transposed weight copies in one launch == per-matrix transposes (ragged 64-tiles)."""
    shapes = [(3072, 1024), (1024, 1024), (520, 136), (64, 4096)]
    srcs = [torch.randn(r, c, device="cuda").bfloat16() for r, c in shapes]
    dsts = [torch.empty(c, r, device="cuda", dtype=torch.bfloat16) for r, c in shapes]
    rows, tiles = [], 0
    for s_, d_ in zip(srcs, dsts):
        R, C = s_.shape
        ntc = -(-C // 64)
        rows.append([s_.data_ptr(), d_.data_ptr(), R, C, tiles, ntc])
        tiles += ntc * -(-R // 64)
    ext.transpose_bf16_batch(torch.tensor(rows, dtype=torch.int64).cuda(), tiles)
    for s_, d_ in zip(srcs, dsts):
        assert torch.equal(d_, s_.t())


def test_weight_t_batched_refresh():
    """ParamStore refreshes every transposed copy in one batch after a shadow update."""
    from jumbo_mae_tpu_amd.config import ViTConfig
    from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
    vc = ViTConfig(layers=2, dim=128, heads=4, labels=10, image_size=32, patch_size=16, posemb="sincos2d")
    m = FinetuneModel(vc).to("cuda", torch.bfloat16, seed=0)
    hs = [h for h in m.store._handles if len(h.shape) == 2 and h.shape[0] % 8 == 0 and h.shape[1] % 8 == 0]
    for h in hs:
        h.weight_t()
    m.store.master.mul_(1.5)
    m.store.sync_shadow()
    assert torch.equal(hs[0].weight_t(), hs[0].weight().t())  # triggers the batched refresh
    for h in hs:
        assert h._wt_version == m.store.version
        assert torch.equal(h._wt, h.weight().t())


@pytest.mark.parametrize("M,N,K", [(512, 12288, 3072), (128, 9216, 2304), (257, 200, 192), (3000, 776, 64),
                                   (4095, 392, 320)])
def test_gemm_narrow_epilogues(ext, M, N, K):
    """The 128 x 192 narrow kernel (M < 4096: the jumbo MLP, heads, small batches) with every fused
    epilogue -- bias store, GELU pair, GELU-only, gelu' + gelu (EPI_GELU_D), dGELU and multiply by
    the saved gelu' with the bias-gradient column sums (EPI_DGELU / EPI_DMUL) -- and the fp32 form,
    against fp32 references; ragged M and N (not multiples of 128 / 192)."""
    torch.manual_seed(5)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.1).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    base = x.float() @ w.float().t()
    h_ref = base + b
    o = ext.gemm_nt(x, w, b, False)[0]
    assert rel(o, h_ref) < 1e-2
    h, gl = ext.gemm_nt(x, w, b, True)
    assert rel(h, h_ref) < 1e-2
    gref = torch.nn.functional.gelu(h.float(), approximate="tanh")
    assert rel(gl, gref) < 1e-2
    go = ext.gemm_nt(x, w, b, True, True)[0]
    assert rel(go, gref) < 1e-2
    gd, g2 = ext.gemm_nt(x, w, b, True, False, True)
    hr = h.float()
    t = torch.tanh(0.7978845608028654 * (hr + 0.044715 * hr ** 3))
    d = 0.5 * (1 + t) + 0.5 * hr * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * hr * hr)
    _gd_check(gd, d)
    assert rel(g2, gref) < 1e-2
    f = ext.gemm_nt_f32(x, w)
    assert f.dtype == torch.float32 and rel(f, base) < 1e-5
    pre = (torch.randn(M, N, device="cuda") * 2).bfloat16()
    codes = torch.randint(0, 256, (M, N), device="cuda", dtype=torch.uint8)
    from jumbo_mae_tpu_amd.ops import prims as P
    for deriv in (False, True):
        db = torch.full((N,), 0.5, device="cuda")
        out = ext.gemm_nt_dgelu(x, w, codes if deriv else pre, db, deriv)
        p = pre.float()
        if deriv:
            mul = P.gd_decode(codes, dtype=torch.float32)
        else:
            tt = torch.tanh(0.7978845608028654 * (p + 0.044715 * p ** 3))
            mul = 0.5 * (1 + tt) + 0.5 * p * (1 - tt * tt) * 0.7978845608028654 * (1 + 3 * 0.044715 * p * p)
        ref = base.bfloat16().float() * mul
        assert rel(out, ref) < 1e-2, deriv
        assert rel(db - 0.5, ref.sum(0)) < 1e-2, deriv


def test_small_m_routing_uses_mfma(ext):
    """Below 4096 rows every Dense forward / data gradient / weight gradient of the prims takes a
    hand-written kernel (no hipBLASLt): fused narrow GEMMs where 160+ tiles fill the chip, split-K
    narrow GEMMs otherwise, a padded reduction for the 1000-class head's data gradient."""
    from jumbo_mae_tpu_amd.ops import prims as P
    assert P.use_our_gemm(512, 12288, 3072, fused_gelu=True) and P.splitk_plan(512, 12288, 3072) == 0
    # K = 12288 jumbo GEMMs: 64 narrow tiles x 4 splits
    assert P.splitk_plan(512, 3072, 12288) == 4
    assert not P.use_our_gemm(128, 9216, 2304, fused_gelu=True) and P.splitk_plan(128, 9216, 2304) >= 2
    from jumbo_mae_tpu_amd.models.params import ParamStore, trunc_normal_t, zeros_
    st = ParamStore()
    hw = st.handle(st.add(("k",), (1000, 768), trunc_normal_t(0.02)))
    hb = st.handle(st.add(("b",), (1000,), zeros_))
    st.finalize("cuda", torch.bfloat16)
    x = torch.randn(96, 768, device="cuda").bfloat16()
    dy = torch.randn(96, 1000, device="cuda").bfloat16()
    y = P.linear_fwd(x, hw, hb)
    w = st.master[:1000 * 768].view(1000, 768)
    assert rel(y, x.float() @ w.bfloat16().float().t()) < 1e-2
    dx = P.linear_bwd(dy, x, hw, hb)
    assert rel(dx, dy.float() @ w.bfloat16().float()) < 1e-2
    assert rel(hw.grad, dy.float().t() @ x.float()) < 1e-2

