"""Host-side logic of the product path that needs no GPU."""
import torch


def test_host_scalar_cache_per_parameter():
    """unrolledswin._host_scalar caches float(p) on the parameter itself, keyed
    by (storage, in-place version): a new parameter never sees another one's
    value, even at a reused address, and an in-place update is picked up."""
    from dl_cs.models.unrolledswin import _host_scalar
    p = torch.nn.Parameter(torch.tensor([-2.0]), requires_grad=False)
    assert _host_scalar(p) == -2.0
    with torch.no_grad():
        p.fill_(0.5)
    assert _host_scalar(p) == 0.5
    q = torch.nn.Parameter(torch.tensor([0.1]), requires_grad=False)
    assert abs(_host_scalar(q) - 0.1) < 1e-7
    assert _host_scalar(p) == 0.5
    p.data = torch.tensor([3.0])
    assert _host_scalar(p) == 3.0
