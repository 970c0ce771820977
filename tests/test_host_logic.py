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


def test_dw_grouped_ok_shapes(monkeypatch):
    """_ops.dw_grouped_ok: the fp32 x6 grouped dW takes M, N multiples of 16 (edge
    tiles: the DiT / Latte widths), bf16 and the DLCS_DW_F32=1 build whole 160
    tiles; tokens a multiple of 64; dense 2-D rows only."""
    from dl_cs.models import _ops as K
    f = lambda *s: torch.zeros(s, dtype=torch.float32)           # noqa: E731
    b = lambda *s: torch.zeros(s, dtype=torch.bfloat16)          # noqa: E731
    assert K.dw_grouped_ok(128, [(f(128, 384), f(128, 1152))])
    assert K.dw_grouped_ok(128, [(f(128, 160), f(128, 640))])
    assert not K.dw_grouped_ok(100, [(f(100, 160), f(100, 160))])          # tokens % 64
    assert not K.dw_grouped_ok(128, [(f(128, 392), f(128, 384))])          # 392 % 16 != 0
    assert not K.dw_grouped_ok(128, [(b(128, 384), b(128, 384))])          # bf16: whole tiles
    assert K.dw_grouped_ok(128, [(b(128, 320), b(128, 160))])
    assert not K.dw_grouped_ok(128, [(f(128, 320)[:, :160], f(128, 160))])  # strided rows
    assert not K.dw_grouped_ok(128, [(f(128, 160), b(128, 160))])          # mixed dtypes
    monkeypatch.setenv("DLCS_DIAG", "1")
    monkeypatch.setenv("DLCS_DW_F32", "1")
    assert not K.dw_grouped_ok(128, [(f(128, 384), f(128, 384))])
    assert K.dw_grouped_ok(128, [(f(128, 320), f(128, 160))])

