"""Per-point head kernels (csrc/head.hip) against fp64 / torch.

rows_wgrad_bf16 returns bf16 (autocast's mm dtype): tolerance = one bf16
rounding (2^-8 relative) of the fp32 sum plus fp32 summation-order noise,
written as |err| <= 2^-8 |ref| + 1e-4 max|ref|."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from pcfm import _lib, ops
    _lib.load()
    return ops


def _check_bf16_sum(out, ref):
    ref = ref.double().cpu()
    err = (out.double().cpu() - ref).abs()
    bound = 2.0 ** -8 * ref.abs() + 1e-4 * ref.abs().max()
    assert bool((err <= bound).all()), float((err - bound).max())


@pytest.mark.parametrize("rows,m,n", [(160000, 512, 512), (5000, 512, 512), (4097, 256, 384),
                                      (3001, 6, 512), (2500, 128, 6), (1000, 512, 326),
                                      (63, 128, 128), (1, 3, 5)])
def test_rows_wgrad_vs_fp64(ops, rows, m, n):
    g = torch.Generator(device="cuda").manual_seed(rows + 3 * m + n)
    a = torch.randn(rows, m, device="cuda", generator=g).bfloat16()
    b = torch.randn(rows, n, device="cuda", generator=g).bfloat16()
    out = ops.rows_wgrad_bf16(a, b)
    assert out.dtype == torch.bfloat16 and out.shape == (m, n)
    _check_bf16_sum(out, a.double().t() @ b.double())


def test_rows_wgrad_strided_rows(ops):
    """A column slice of a wider tensor (row stride > width), as autograd can hand in."""
    g = torch.Generator(device="cuda").manual_seed(5)
    wide = torch.randn(7000, 520, device="cuda", generator=g).bfloat16()
    a = wide[:, :512]
    b = torch.randn(7000, 131, device="cuda", generator=g).bfloat16()
    _check_bf16_sum(ops.rows_wgrad_bf16(a, b), a.double().t() @ b.double())


def test_rows_wgrad_deterministic(ops):
    g = torch.Generator(device="cuda").manual_seed(9)
    a = torch.randn(50000, 512, device="cuda", generator=g).bfloat16()
    b = torch.randn(50000, 512, device="cuda", generator=g).bfloat16()
    assert torch.equal(ops.rows_wgrad_bf16(a, b), ops.rows_wgrad_bf16(a, b))


def test_rows_wgrad_zero_rows(ops):
    a = torch.empty(0, 8, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(0, 4, device="cuda", dtype=torch.bfloat16)
    assert torch.count_nonzero(ops.rows_wgrad_bf16(a, b)) == 0


@pytest.mark.parametrize("shape,fin,fout", [((8, 2000, 326), 326, 512), ((16000, 512), 512, 512),
                                            ((8, 2000, 6), 6, 128), ((16000, 512), 512, 6)])
def test_rows_linear_matches_linear_under_autocast(ops, shape, fin, fout):
    from pcfm.layers import RowsLinear
    torch.manual_seed(0)
    ref = torch.nn.Linear(fin, fout).cuda()
    mod = RowsLinear(fin, fout).cuda()
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(*shape, device="cuda")
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ya, yb = ref(xa), mod(xb)
    assert ya.dtype == yb.dtype == torch.bfloat16
    assert torch.equal(ya, yb)  # same library GEMM forward
    gy = torch.randn_like(ya)
    ya.backward(gy)
    yb.backward(gy)
    torch.testing.assert_close(xb.grad, xa.grad, rtol=2 ** -7, atol=1e-3)
    # weight grad: the bf16 rounding of the fp32 sum of bf16 products
    g64 = gy.double().reshape(-1, fout)
    x64 = x.bfloat16().double().reshape(-1, fin)
    _check_bf16_sum(mod.weight.grad, g64.t() @ x64)
    torch.testing.assert_close(mod.bias.grad, ref.bias.grad, rtol=2 ** -7, atol=1e-2)


def test_rows_linear_plain_outside_autocast(ops):
    from pcfm.layers import RowsLinear
    mod = RowsLinear(16, 8).cuda()
    x = torch.randn(5000, 16, device="cuda")
    torch.testing.assert_close(mod(x), torch.nn.functional.linear(x, mod.weight, mod.bias))


def _relnorm(a, b):
    a, b = a.detach().double(), b.detach().double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("width,n", [(512, 3000), (256, 777)])
def test_fused_trunk_matches_torch_trunk(ops, width, n):
    """VelocityNetWithContext under bf16 autocast: the fused trunk (csrc/head_film.hip
    + library GEMMs + rows_wgrad) against the module's own torch path.  Both round
    at the same points (bf16 Linear outputs and inputs); what differs is fp32
    summation order, so a bf16 rounding can flip: relative-norm tolerance 1e-2."""
    from pcfm.models import VelocityNetWithContext
    torch.manual_seed(1)
    b = 2
    net = VelocityNetWithContext(cond_dim=129, point_dim=6, ctx_dim=64, width=width, depth=6,
                                 emb_dim=256).cuda()
    # non-trivial LayerNorm affine and FiLM so every gradient path is exercised
    with torch.no_grad():
        for film in net.films:
            film.norm.weight.normal_(1.0, 0.2)
            film.norm.bias.normal_(0.0, 0.2)
            film.affine.weight.normal_(0.0, 0.05)
        net.out[1].weight.normal_(0.0, 0.05)
    x = torch.randn(b, n, 6, device="cuda")
    ctx = torch.randn(b, n, 64, device="cuda")
    t = torch.rand(b, device="cuda")
    cond = torch.randn(b, 129, device="cuda")
    gy = torch.randn(b, n, 6, device="cuda")
    res = []
    for fused in (False, True):
        net.fused = fused
        net.zero_grad(set_to_none=True)
        xx, cc = x.clone().requires_grad_(True), ctx.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            v = net(xx, t, cond, cc)
        (v.float() * gy).sum().backward()
        grads = {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None}
        res.append((v.detach(), xx.grad, cc.grad, grads))
    (v0, gx0, gc0, g0), (v1, gx1, gc1, g1) = res
    assert v1.dtype == v0.dtype == torch.bfloat16
    assert _relnorm(v1, v0) < 1e-2
    assert _relnorm(gx1, gx0) < 1e-2 and _relnorm(gc1, gc0) < 1e-2
    assert set(g0) == set(g1)
    for k in g0:
        assert _relnorm(g1[k], g0[k]) < 2e-2, k


@pytest.mark.parametrize("w,first", [(512, False), (512, True), (256, False)])
def test_film_bwd_recomputed_u_is_bitwise(ops, w, first):
    """pcfm_head_film_bwd with u = NULL (recomputed from h, the row statistics and
    shift) returns exactly what it returns when handed the forward's u."""
    b, n = 3, 1000
    g = torch.Generator(device="cuda").manual_seed(w + first)
    rnd = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    gamma, beta = 1.0 + 0.2 * rnd(w), 0.2 * rnd(w)
    sp1, sh = (1.0 + 0.1 * rnd(b, w)).bfloat16(), (0.1 * rnd(b, w)).bfloat16()
    if first:
        h16, hb, uprev, gprev = rnd(b * n, w).bfloat16(), rnd(b, w), None, None
    else:
        h16, hb, uprev, gprev = None, None, rnd(b * n, w), rnd(b * n, w).bfloat16()
    u, a, mean, rstd = ops.head_film_fwd(h16, uprev, gprev, gamma, beta, sp1, sh, n, 1e-5,
                                         hbias=hb)
    dhn, da = rnd(b * n, w), rnd(b * n, w).bfloat16()
    r0 = ops.head_film_bwd(dhn, da, u, h16, uprev, gprev, mean, rstd, gamma, beta, sp1, n,
                           want_dh=True, hbias=hb)
    r1 = ops.head_film_bwd(dhn, da, None, h16, uprev, gprev, mean, rstd, gamma, beta, sp1, n,
                           want_dh=True, hbias=hb, shift=sh)
    assert len(r0) == len(r1)
    for x0, x1 in zip(r0, r1):
        assert torch.equal(x0, x1)


@pytest.mark.parametrize("b,n,c", [(8, 20000, 128), (2, 777, 6), (3, 50, 384)])
def test_rows_max_matches_torch(ops, b, n, c):
    from pcfm.layers import max_over_points
    g = torch.Generator(device="cuda").manual_seed(n + c)
    h = torch.randn(b, n, c, device="cuda", generator=g).bfloat16()
    h[0, 5:9, 0] = 100.0  # a tie: the lowest index wins
    val, idx = ops.rows_max_bf16(h)
    ref = h.max(dim=1).values
    assert torch.equal(val, ref)
    assert int(idx[0, 0]) == 5
    assert torch.equal(h.gather(1, idx.long().unsqueeze(1)).squeeze(1), ref)
    hh = h.clone().requires_grad_(True)
    v = max_over_points(hh)
    gv = torch.randn_like(v)
    v.backward(gv)
    exp = torch.zeros_like(h).scatter_(1, idx.long().unsqueeze(1), gv.unsqueeze(1))
    assert torch.equal(hh.grad, exp)


@pytest.mark.parametrize("shape,dtype", [((160000, 128), torch.bfloat16), ((8, 20000, 64), torch.float32),
                                         ((3, 777, 6), torch.bfloat16), ((1, 5, 512), torch.float32)])
def test_rows_colsum_matches_sum(ops, shape, dtype):
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    x = torch.randn(*shape, device="cuda", generator=g).to(dtype)
    got = ops.rows_colsum(x)
    want = x.double().sum(dim=-2)
    scale = x.double().abs().sum(dim=-2).max()
    assert got.shape == want.shape and got.dtype == torch.float32
    assert ((got.double() - want).abs().max() / scale).item() < 1e-6
    assert torch.equal(ops.rows_colsum(x), got)  # deterministic


def test_tgate_matches_torch(ops):
    from pcfm.models import _TGate
    g = torch.Generator(device="cuda").manual_seed(3)
    b, c, n = 3, 64, 1000
    head = torch.randn(b, c, n, device="cuda", generator=g).requires_grad_(True)
    glb = torch.randn(b, c, device="cuda", generator=g).requires_grad_(True)
    alpha = torch.rand(b, device="cuda", generator=g)
    out = _TGate.apply(head, glb, alpha)
    ref_h = head.detach().double().requires_grad_(True)
    ref_g = glb.detach().double().requires_grad_(True)
    a = alpha.double().view(b, 1, 1)
    ref = a * ref_h.permute(0, 2, 1) + (1.0 - a) * ref_g[:, None, :].expand(b, n, c)
    assert out.shape == (b, n, c) and out.is_contiguous()
    assert (out.double() - ref).abs().max().item() < 1e-5
    gy = torch.randn(b, n, c, device="cuda", generator=g)
    dh, dg = torch.autograd.grad(out, [head, glb], gy)
    rh, rg = torch.autograd.grad(ref, [ref_h, ref_g], gy.double())
    assert (dh.double() - rh).abs().max().item() < 1e-5
    assert ((dg.double() - rg).abs().max() / rg.abs().max()).item() < 1e-5
