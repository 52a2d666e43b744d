"""The oracle's teacher-forced activation decisions (oracle.ActDecisions, used by the GPU parity
tests to compare gradients at full size) are exact: forcing a network's OWN decisions -- handed
over channels-last-strided, as the HIP path's NHWC buffers produce them -- reproduces its free
forward and backward exactly (G + D, smooth loss), and a forced flip is logged with its kink
distance."""
import torch
import torch.nn.functional as F

import oracle.paired_attention as P
from oracle import paired_attention as O


def _record(Gp, Dp, x):
    rec, cur = {"G": {}, "D": {}}, [None]
    orig = P._act

    def spy(h, slope, name, forced):
        # NHWC-strided, like floodgan.executor's decisions
        rec[cur[0]][name] = (h.detach() > 0).permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)
        return orig(h, slope, name, None)
    P._act = spy
    try:
        with torch.no_grad():
            cur[0] = "G"
            fake, _ = O.generator_forward(Gp, x)
            cur[0] = "D"
            O.discriminator_forward(Dp, torch.cat((x, fake), 1))
    finally:
        P._act = orig
    return {"G": [rec["G"]], "D": [rec["D"]]}


def _grads(Gp, Dp, x, y, dec):
    Gd = {k: v.double().requires_grad_(True) for k, v in Gp.items()}
    Dd = {k: v.double().requires_grad_(True) for k, v in Dp.items()}
    fake, _ = O.generator_forward(Gd, x.double(), O._forced(dec, "G"))
    pr = O.discriminator_forward(Dd, torch.cat((x.double(), fake), 1), O._forced(dec, "D"))
    (F.mse_loss(pr, torch.ones_like(pr)) + 100 * F.mse_loss(fake, y.double())).backward()
    return {**{k: v.grad for k, v in Gd.items()}, **{"D." + k: v.grad for k, v in Dd.items()}}


def test_forced_own_decisions_reproduce_free_gradients():
    torch.manual_seed(3)
    x = torch.rand(1, 9, 32, 32) * 2 - 1
    y = torch.rand(1, 3, 32, 32) * 2 - 1
    Gp, Dp = O.init_params()
    masks = _record({k: v.double() for k, v in Gp.items()}, {k: v.double() for k, v in Dp.items()}, x.double())
    dec = O.ActDecisions(masks)
    forced = _grads(Gp, Dp, x, y, dec)
    free = _grads(Gp, Dp, x, y, None)
    assert sum(n for _, _, n, _ in dec.log) == 0
    for k in free:
        assert torch.allclose(forced[k], free[k], rtol=1e-12, atol=1e-300), k


def test_forced_flip_is_logged():
    torch.manual_seed(4)
    x = torch.rand(1, 9, 32, 32) * 2 - 1
    Gp, Dp = O.init_params()
    masks = _record(Gp, Dp, x)
    m = masks["G"][0]["block3"].clone()
    m[0, 5, 2, 2] = ~m[0, 5, 2, 2]
    masks["G"][0]["block3"] = m
    dec = O.ActDecisions(masks)
    with torch.no_grad():
        O.generator_forward(Gp, x, O._forced(dec, "G"))
    flips = [(layer, n) for _, layer, n, _ in dec.log if n]
    # the forced flip is the first disagreement; later layers see its effect on their own inputs
    assert flips[0] == ("block3", 1) and dec.worst() > 0
    assert [layer for _, layer, _, _ in dec.log].index("block3") == 6
