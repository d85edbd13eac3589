"""Host-side hand-off of the fused norm-backward / bias partials (ops/hip.py).

The GPU tests (tests/test_nb_fuse_gpu.py) check the numerics; this pins the bookkeeping that
decides WHEN the fused partials may be used, on plain CPU tensors:
  * a norm output is found only as the very tensor the norm returned (not a view or copy);
  * parked partials are taken only by exactly the gradient tensor they were computed from
    (an autograd-accumulated gradient is a new tensor -> the norm runs its own partial pass);
  * which input half of a conv may carry them (never a deferred skip half; a "take" half only
    when its parked gradient is added in the epilogue);
  * begin_step() drops everything (a backward that raised part-way leaks nothing).
"""
import torch

from p2p_pytorch_amd.ops import hip


class _Cfg:
    def __init__(self, skip_grad=None):
        self.skip_grad = skip_grad


def test_norm_output_lookup_is_identity_based():
    hip.begin_step()
    z = torch.randn(2, 8, 4, 4)
    info = ("x", "mean", "rstd", None, None, 2, False, None)
    hip._register_norm_out(z, info)
    assert hip._norm_lookup(z) is info
    assert hip._norm_lookup(z.view(2, 8, 4, 4)) is None       # same storage, other object
    assert hip._norm_lookup(z.clone()) is None
    assert hip._norm_lookup(None) is None
    hip.begin_step()
    assert hip._norm_lookup(z) is None


def test_parked_partials_taken_only_by_the_same_gradient():
    hip.begin_step()
    g = torch.randn(2, 8, 4, 4)
    parts = torch.zeros(2, 2, 1, 8)
    hip._stash_nbp(g, parts)
    assert hip._take_nbp(g.clone()) is None
    hip._stash_nbp(g, parts)
    assert hip._take_nbp(g + 0) is None                     # accumulated gradient: new tensor
    hip._stash_nbp(g, parts)
    assert hip._take_nbp(g) is parts
    assert hip._take_nbp(g) is None                         # taken once
    hip._stash_nbp(g, parts)
    hip.begin_step()
    assert not hip._nbp_stash


def test_which_half_carries_the_partials():
    n1, n2 = ("n1",), ("n2",)
    q2 = torch.zeros(1)
    assert hip._nb_half(_Cfg(), None, None, True) is None
    assert hip._nb_half(_Cfg(), None, (n1, None), False) == (1, n1)
    # a deferred skip half is only part of its tensor's gradient
    assert hip._nb_half(_Cfg("defer"), q2, (n1, n2), True) == (2, n2)
    assert hip._nb_half(_Cfg("defer"), None, (n1, None), True) is None
    # "take": complete only when the parked gradient is fused into this epilogue
    assert hip._nb_half(_Cfg("take"), None, (n1, None), True) == (1, n1)
    assert hip._nb_half(_Cfg("take"), None, (n1, None), False) is None
    assert hip._nb_half(_Cfg(), q2, (None, n2), False) == (2, n2)


def test_nb_kwargs_modes():
    assert hip._nb_kwargs(None) == {}
    assert hip._nb_kwargs((1, hip._CS)) == {"nb_half": 1, "nb_colsum": True}
    kw = hip._nb_kwargs((2, ("x", "m", "r", None, None, 1, True, None)))
    assert kw["nb_half"] == 2 and kw["nb_act"] == 1 and kw["nb_batch"] is True and kw["nb_x"] == "x"
    assert kw["nb_prelu"] is None and kw["nb_gate"] is False
    # affine batch norm with a shared-slope PReLU (family R): slope handed over, no xhat gate
    kw = hip._nb_kwargs((1, ("x", "m", "r", "g", "b", 0, True, "w")))
    assert kw["nb_prelu"] == "w" and kw["nb_gamma"] == "g" and kw["nb_gate"] is False
