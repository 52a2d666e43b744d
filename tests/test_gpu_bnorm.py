"""BatchNorm (training mode) kernels of csrc/bnorm.hip vs torch-CPU fp64 (nn.BatchNorm2d semantics,
models/model_architectures.py:34-35, :74-80): batch statistics per group of images (the reference's
separate D(fake) / D(real) calls fused into one pass), running statistics updated once per group in
order, the affine transform, Dropout with a given mask (x mask / 0.5), two differently activated
outputs written into a padded buffer and a channel slice of a wider one (the U-Net's cat halves), the
backward through both activations, the dropout and the group statistics; nn.MaxPool2d(2)."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_parity import DEV, KTOL, buf_from, nchw, nrel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _ref_fwd(x, groups, gamma, beta, rm, rv, mask):
    """fp64 CPU: sequential BN calls per group (F.batch_norm updates rm / rv in place)"""
    outs = []
    for xg in x.chunk(groups, 0):
        outs.append(F.batch_norm(xg, rm, rv, gamma, beta, training=True, momentum=0.1, eps=1e-5))
    u = torch.cat(outs, 0)
    return u * (mask / 0.5) if mask is not None else u


CASES = [(2, 64, 8, 8, 1, False), (4, 128, 16, 12, 2, True), (2, 512, 1, 1, 1, False), (2, 512, 2, 2, 1, True),
         (6, 256, 4, 4, 3, False), (1, 64, 64, 64, 1, True), (8, 64, 64, 64, 2, True)]


@pytest.mark.parametrize("n,c,h,w,groups,drop", CASES)
def test_bn_forward_backward(n, c, h, w, groups, drop):
    from floodgan import _lib as L
    from floodgan import ops
    from floodgan.plans import Buf, Slice

    g = torch.Generator().manual_seed(n * 1000 + c + h)
    x = torch.randn(n, c, h, w, generator=g, dtype=torch.float64) * 1.7 + 0.6
    gamma = 1 + 0.1 * torch.randn(c, generator=g, dtype=torch.float64)
    beta = 0.1 * torch.randn(c, generator=g, dtype=torch.float64)
    rm0, rv0 = 0.3 * torch.randn(c, generator=g, dtype=torch.float64), 1 + torch.rand(c, generator=g, dtype=torch.float64)
    mask = torch.empty(n, c, h, w, dtype=torch.float32).bernoulli_(0.5, generator=g) if drop else None
    gA = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)
    gB = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)

    # fp64 reference with autograd
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gamma, beta))
    rm, rv = rm0.clone(), rv0.clone()
    u = _ref_fwd(xr, groups, gr, br, rm, rv, None if mask is None else mask.double())
    yA, yB = F.leaky_relu(u, 0.2), F.relu(u)
    dx, dgam, dbet = torch.autograd.grad((yA * gA).sum() + (yB * gB).sum(), (xr, gr, br))

    # HIP
    src = buf_from(x, 0, "constant")
    dA = Buf.zeros(n, h, w, c, 1, DEV)
    wide = Buf.zeros(n, h, w, 2 * c, 0, DEV)
    d_gamma, d_beta = gamma.float().to(DEV), beta.float().to(DEV)
    d_rm, d_rv = rm0.float().to(DEV), rv0.float().to(DEV)
    d_mask = mask.to(DEV) if mask is not None else None
    mean, invstd = ops.bn_stats(src, groups, (d_rm, d_rv))
    ops.bn_apply(src, groups, mean, invstd, d_gamma, d_beta, d_mask, L.FG_ACT_LRELU, dA, L.FG_ACT_RELU,
                 Slice(wide, c, c))
    torch.cuda.synchronize()
    assert nrel(nchw(dA), yA) < KTOL
    assert nrel(wide.interior()[..., c:].permute(0, 3, 1, 2).cpu(), yB) < KTOL
    assert float(wide.interior()[..., :c].abs().max()) == 0.0            # the other half untouched
    assert float(dA.nhwc()[:, 0].abs().max()) == 0.0                      # border untouched
    assert nrel(d_rm.cpu(), rm) < KTOL and nrel(d_rv.cpu(), rv) < KTOL

    # backward: gA through LeakyReLU, gB (a channel slice) through ReLU
    gAb = buf_from(gA, 0, "constant")
    gwide = buf_from(torch.cat((torch.zeros_like(gB), gB), 1), 0, "constant")
    dst = Buf.zeros(n, h, w, c, 1, DEV)
    gg, gb = torch.zeros(c, device=DEV), torch.full((c,), 5.0, device=DEV)
    ops.bn_bwd(gAb, L.FG_ACT_LRELU, Slice(gwide, c, c), L.FG_ACT_RELU, src, groups, mean, invstd, d_gamma, d_beta,
               d_mask, dst, gg, gb, accumulate=False)
    torch.cuda.synchronize()
    assert nrel(nchw(dst), dx) < KTOL
    assert nrel(gg.cpu(), dgam) < KTOL and nrel(gb.cpu(), dbet) < KTOL
    # accumulate adds onto the existing gradients
    ops.bn_bwd(gAb, L.FG_ACT_LRELU, Slice(gwide, c, c), L.FG_ACT_RELU, src, groups, mean, invstd, d_gamma, d_beta,
               d_mask, dst, gg, gb, accumulate=True)
    torch.cuda.synchronize()
    assert nrel(gg.cpu(), 2 * dgam) < KTOL and nrel(gb.cpu(), 2 * dbet) < KTOL


def test_bn_identity_mode_and_large_mean():
    """mean=None: activation only (the U-Net's un-normalised outermost / innermost downs); a channel
    whose mean dwarfs its spread (shifted sums keep the variance accurate)"""
    from floodgan import _lib as L
    from floodgan import ops
    from floodgan.plans import Buf

    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 32, 32, generator=g, dtype=torch.float64)
    src = buf_from(x, 0, "constant")
    d0, d1 = Buf.zeros(2, 32, 32, 64, 1, DEV), Buf.zeros(2, 32, 32, 64, 1, DEV)
    ops.bn_apply(src, 1, None, None, None, None, None, L.FG_ACT_LRELU, d0, L.FG_ACT_RELU, d1)
    torch.cuda.synchronize()
    assert nrel(nchw(d0), F.leaky_relu(x, 0.2)) < KTOL and nrel(nchw(d1), F.relu(x)) < KTOL
    gA = torch.randn(2, 64, 32, 32, generator=g, dtype=torch.float64)
    dst = Buf.zeros(2, 32, 32, 64, 1, DEV)
    ops.bn_bwd(buf_from(gA, 0, "constant"), L.FG_ACT_RELU, None, 0, src, 1, None, None, None, None, None, dst)
    torch.cuda.synchronize()
    assert nrel(nchw(dst), gA * (x > 0)) < KTOL

    xb = x * 0.01 + 300.0
    srcb = buf_from(xb, 0, "constant")
    mean, invstd = ops.bn_stats(srcb, 1)
    torch.cuda.synchronize()
    var = xb.var(dim=(0, 2, 3), unbiased=False)
    assert nrel(mean.cpu(), xb.mean(dim=(0, 2, 3))) < 1e-7
    assert nrel(invstd.cpu(), 1 / torch.sqrt(var + 1e-5)) < 1e-4


@pytest.mark.parametrize("h,w", [(16, 16), (7, 9), (2, 2)])
def test_maxpool2(h, w):
    from floodgan import ops
    from floodgan.plans import Buf

    x = torch.randn(3, 128, h, w, dtype=torch.float64, generator=torch.Generator().manual_seed(h * w))
    dst = Buf.zeros(3, h // 2, w // 2, 128, 1, DEV)
    ops.maxpool2(buf_from(x, 1, "constant"), dst)
    torch.cuda.synchronize()
    assert torch.equal(nchw(dst).double(), F.max_pool2d(x.float(), 2).double())


def test_hashed_dropout_equals_its_mask():
    """Device dropout (keep decisions hashed from (seed, NCHW index), recomputed in the backward) gives
    exactly the result of the same decisions passed as a mask; the decisions are Bernoulli(0.5):
    the kept fraction and its independence across seeds / neighbouring elements."""
    from floodgan import _lib as L
    from floodgan import ops
    from floodgan.plans import Buf

    g = torch.Generator().manual_seed(11)
    n, c, h, w = 2, 512, 16, 16
    x = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)
    gA = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)
    gamma, beta = torch.ones(c, device=DEV), torch.zeros(c, device=DEV)
    src = buf_from(x, 0, "constant")
    seed = 0x1234_5678_9ABC
    mask = ops.dropout_mask(seed, (n, c, h, w), DEV)
    outs = []
    for drop in (seed, mask):
        mean, invstd = ops.bn_stats(src, 1)
        d = Buf.zeros(n, h, w, c, 1, DEV)
        ops.bn_apply(src, 1, mean, invstd, gamma, beta, drop, L.FG_ACT_RELU, d)
        gd = Buf.zeros(n, h, w, c, 1, DEV)
        ops.bn_bwd(buf_from(gA, 0, "constant"), L.FG_ACT_RELU, None, 0, src, 1, mean, invstd, gamma, beta, drop, gd)
        torch.cuda.synchronize()
        outs.append((nchw(d), nchw(gd)))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    m = mask.cpu().double()
    assert set(m.unique().tolist()) == {0.0, 1.0}
    assert abs(float(m.mean()) - 0.5) < 0.005                                # 262144 draws: sd 0.001
    m2 = ops.dropout_mask(seed + 1, (n, c, h, w), DEV).cpu().double()
    assert abs(float(((m - 0.5) * (m2 - 0.5)).mean())) < 0.005              # seeds independent
    assert abs(float(((m[..., 1:] - 0.5) * (m[..., :-1] - 0.5)).mean())) < 0.005   # neighbours independent
