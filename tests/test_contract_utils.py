"""Training-utility contracts K13-K18 (softmax, cross-entropy, clipping, AdamW,
cosine LR, get_batch, checkpointing).  Expected values are the reference's
(``tests/test_nn_utils.py``, ``test_optimizer.py``, ``test_data.py``,
``test_serialization.py`` in the reference) or PyTorch's own ops."""

from __future__ import annotations

import io
import math
from collections import Counter

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from .adapters import (
    get_adamw_cls,
    run_cross_entropy,
    run_get_batch,
    run_get_lr_cosine_schedule,
    run_gradient_clipping,
    run_load_checkpoint,
    run_save_checkpoint,
    run_softmax,
)

X5 = torch.tensor([[0.4655, 0.8303, 0.9608, 0.9656, 0.6840], [0.2583, 0.2198, 0.9334, 0.2995, 0.1722],
                   [0.1573, 0.6860, 0.1327, 0.7284, 0.6811]])


@pytest.mark.parametrize("shift", [0.0, 100.0])
def test_softmax_stable(shift):
    torch.testing.assert_close(run_softmax(X5 + shift, dim=-1), F.softmax(X5, dim=-1), atol=1e-6, rtol=0)


def test_softmax_other_dim():
    x = torch.randn(3, 4, 5)
    torch.testing.assert_close(run_softmax(x, 1), F.softmax(x, 1), atol=1e-6, rtol=0)


@pytest.mark.parametrize("scale", [1.0, 1000.0])
def test_cross_entropy(scale):
    g = torch.Generator().manual_seed(0)
    x = scale * torch.rand(8, 5, generator=g)
    t = torch.randint(0, 5, (8,), generator=g)
    torch.testing.assert_close(run_cross_entropy(x, t), F.cross_entropy(x, t), atol=1e-4, rtol=0)


def test_gradient_clipping_matches_torch():
    base = [torch.randn(5, 5) for _ in range(6)]
    a = [torch.nn.Parameter(t.clone()) for t in base]
    b = [torch.nn.Parameter(t.clone()) for t in base]
    a[-1].requires_grad_(False)
    b[-1].requires_grad_(False)
    torch.cat(a).sum().backward()
    torch.cat(b).sum().backward()
    torch.nn.utils.clip_grad_norm_(a, 1e-2)
    run_gradient_clipping(b, 1e-2)
    for pa, pb in zip(a, b):
        if pa.grad is None:
            assert pb.grad is None
        else:
            torch.testing.assert_close(pb.grad, pa.grad, atol=1e-6, rtol=0)


def _optimize(cls):
    torch.manual_seed(42)
    model = torch.nn.Linear(3, 2, bias=False)
    opt = cls(model.parameters(), lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999), eps=1e-8)
    for _ in range(1000):
        opt.zero_grad()
        x = torch.rand(3)
        loss = ((torch.stack([x[0] + x[1], -x[2]]) - model(x)) ** 2).sum()
        loss.backward()
        opt.step()
    return model.weight.detach()


def test_adamw(numpy_snapshot):
    ours = _optimize(get_adamw_cls())
    theirs = _optimize(torch.optim.AdamW)
    torch.testing.assert_close(ours, theirs, atol=1e-4, rtol=0)
    numpy_snapshot.assert_match(ours, atol=1e-4)


def test_cosine_schedule():
    expected = [0, 0.14285714285714285, 0.2857142857142857, 0.42857142857142855, 0.5714285714285714,
                0.7142857142857143, 0.8571428571428571, 1.0, 0.9887175604818206, 0.9554359905560885,
                0.9018241671106134, 0.8305704108364301, 0.7452476826029011, 0.6501344202803414, 0.55,
                0.44986557971965857, 0.3547523173970989, 0.26942958916356996, 0.19817583288938662,
                0.14456400944391146, 0.11128243951817937, 0.1, 0.1, 0.1, 0.1]
    got = [run_get_lr_cosine_schedule(i, 1.0, 0.1, 7, 21) for i in range(25)]
    np.testing.assert_allclose(got, expected)


def test_get_batch_uniform_and_shifted():
    data = np.arange(0, 100)
    ctx, bs, iters = 7, 32, 1000
    starts = Counter()
    for _ in range(iters):
        x, y = run_get_batch(data, bs, ctx, "cpu")
        assert x.shape == (bs, ctx) and y.shape == (bs, ctx) and x.dtype == torch.long
        assert torch.equal(x + 1, y)
        starts.update(x[:, 0].tolist())
    n = len(data) - ctx
    assert min(starts) == 0 and max(starts) == n - 1
    mu = iters * bs / n
    sd = math.sqrt(iters * bs * (1 / n) * (1 - 1 / n))
    assert all(mu - 5 * sd <= c <= mu + 5 * sd for c in starts.values())


def test_get_batch_invalid_device_raises():
    with pytest.raises((RuntimeError, AssertionError)):
        run_get_batch(np.arange(100), 4, 7, "cuda:99")


def test_get_batch_memmap(tmp_path):
    from bpe_transformer.data import load_tokens, write_tokens

    n = write_tokens(range(1000), tmp_path / "toks.bin", vocab_size=50_000)
    mm = load_tokens(tmp_path / "toks.bin", vocab_size=50_000)
    assert n == 1000 and len(mm) == 1000
    x, y = run_get_batch(mm, 8, 16, "cpu")
    assert torch.equal(x + 1, y)


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = torch.nn.Linear(100, 200)
        self.fc2 = torch.nn.Linear(200, 10)

    def forward(self, x):
        return self.fc2(F.relu(self.fc1(x)))


@pytest.mark.parametrize("to_buffer", [False, True])
def test_checkpoint_roundtrip(tmp_path, to_buffer):
    torch.manual_seed(42)
    net, opt = _Net(), None
    opt = get_adamw_cls()(net.parameters(), lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999), eps=1e-8)
    for _ in range(10):
        opt.zero_grad()
        ((net(torch.rand(100)) - torch.rand(10)) ** 2).sum().backward()
        opt.step()
    dst = io.BytesIO() if to_buffer else tmp_path / "ckpt.pt"
    run_save_checkpoint(net, opt, 10, dst)
    if to_buffer:
        dst.seek(0)
    net2 = _Net()
    opt2 = get_adamw_cls()(net2.parameters(), lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999), eps=1e-8)
    assert run_load_checkpoint(dst, net2, opt2) == 10
    for k, v in net.state_dict().items():
        torch.testing.assert_close(net2.state_dict()[k], v, atol=1e-8, rtol=1e-5)
    s1, s2 = opt.state_dict(), opt2.state_dict()
    assert s1["param_groups"] == s2["param_groups"]
    for pid, st in s1["state"].items():
        for key, val in st.items():
            if torch.is_tensor(val):
                torch.testing.assert_close(s2["state"][pid][key], val, atol=1e-8, rtol=1e-5)
            else:
                assert s2["state"][pid][key] == val
