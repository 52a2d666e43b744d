"""torch.library operators of floodgan.custom_ops: schema / fake-tensor / autograd registration
(torch.library.opcheck), results equal to the drop-in modules' (same kernels), and tracing through
torch.compile (aot_eager, fullgraph) with the fake implementations."""
import pytest
import torch

from test_gpu_parity import DEV, nrel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _model():
    from floodgan.model import Model
    return Model(model="PairedAttention", device=DEV)


def test_opcheck_and_equivalence():
    from floodgan import custom_ops  # noqa: F401  (registers the operators)
    from floodgan.model_architectures import DISC_KEYS, GEN_KEYS
    m = _model()
    gp = [m.generator.param_dict()[k] for k in GEN_KEYS]
    dp = [m.discriminator.param_dict()[k] for k in DISC_KEYS]
    g = torch.Generator().manual_seed(4)
    x = (torch.rand((1, 9, 32, 32), generator=g) * 2 - 1).to(DEV)
    xd = (torch.rand((1, 12, 32, 32), generator=g) * 2 - 1).to(DEV)
    torch.library.opcheck(torch.ops.floodgan.paired_attention_generator.default, (x, gp),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))
    torch.library.opcheck(torch.ops.floodgan.patchgan_discriminator.default, (xd, dp),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))
    w, b = torch.randn(64, 9, 7, 7, device=DEV) * 0.02, torch.zeros(64, device=DEV)
    torch.library.opcheck(torch.ops.floodgan.conv2d.default, (x, w, b, 1, 3, True),
                          test_utils=("test_schema", "test_faketensor"))
    # same kernels as the modules: forward and gradients identical
    out, mask = torch.ops.floodgan.paired_attention_generator(x, gp)
    ref = m.generator(x)
    assert torch.equal(out, ref) and torch.equal(mask, m.generator.last_attention_mask)
    xg = x.clone().requires_grad_(True)
    out, _ = torch.ops.floodgan.paired_attention_generator(xg, gp)
    grads = torch.autograd.grad(out.square().sum(), [xg] + gp)
    xr = x.clone().requires_grad_(True)
    ref_grads = torch.autograd.grad(m.generator(xr).square().sum(), [xr] + list(m.generator.param_dict().values()))
    assert max(nrel(a, b) for a, b in zip(grads, ref_grads)) < 1e-6
    # conv2d vs torch fp64
    y = torch.ops.floodgan.conv2d(x, w, b, 1, 3, True)
    yr = torch.nn.functional.conv2d(torch.nn.functional.pad(x.double(), (3,) * 4, mode="reflect"), w.double(),
                                    b.double())
    assert nrel(y, yr) < 1e-5


def test_compile_traces_through_custom_ops():
    from floodgan import custom_ops  # noqa: F401
    from floodgan.model_architectures import GEN_KEYS
    m = _model()
    gp = [m.generator.param_dict()[k] for k in GEN_KEYS]
    x = torch.rand((1, 9, 32, 32), device=DEV) * 2 - 1

    def f(x, ps):
        out, mask = torch.ops.floodgan.paired_attention_generator(x, ps)
        return out.mean() + mask.mean()

    got = torch.compile(f, backend="aot_eager", fullgraph=True)(x, gp)
    assert torch.allclose(got, f(x, gp))


def test_backward_without_materialized_mask_grad():
    """the generator operator's backward formula with dL/dmask = None (autograd with materialize_grads off)
    equals the one with a zero mask gradient (an empty tensor is passed to the Tensor-typed schema)"""
    from types import SimpleNamespace

    from floodgan import custom_ops
    from floodgan.model_architectures import GEN_KEYS
    m = _model()
    gp = [m.generator.param_dict()[k] for k in GEN_KEYS]
    g = torch.Generator().manual_seed(5)
    x = (torch.rand((1, 9, 32, 32), generator=g) * 2 - 1).to(DEV)
    g_out = torch.rand((1, 3, 32, 32), generator=g).to(DEV)
    ctx = SimpleNamespace(saved_tensors=(x, *gp))
    gx0, gp0 = custom_ops._gen_backward(ctx, g_out, None)
    gx1, gp1 = custom_ops._gen_backward(ctx, g_out, torch.zeros((1, 32, 32), device=DEV))
    assert torch.equal(gx0, gx1) and all(torch.equal(a, b) for a, b in zip(gp0, gp1))
