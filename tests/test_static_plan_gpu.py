"""``ops.static_plan`` (``table_ops.hip`` ``static_plan_kernel``): the world-1 static
de-duplicated plan in one launch equals the torch expression it replaced
(``parallel/tensor_ps.py``: real keys first, padding slot j -> uniq[j mod U])."""
import pytest
import torch

from flink_parameter_server_1_amd import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("n,U,nb", [(4096, 1500, 4096), (4096, 4096, 4096), (300, 0, 300), (5000, 17, 2000),
                                    (1, 1, 1)])
def test_static_plan_equals_torch(n, U, nb):
    g = torch.Generator(device=DEV).manual_seed(n + U)
    uniq = torch.randint(0, 10**6, (max(n, nb),), generator=g, device=DEV, dtype=torch.int32)
    prefix = torch.tensor([0, U], dtype=torch.int32, device=DEV)
    pos = torch.randint(0, max(U, 1), (n,), generator=g, device=DEV, dtype=torch.int32)
    gk, va, pc, pr = ops.static_plan(uniq, prefix, nb, pos)
    j = torch.arange(nb, device=DEV)
    valid = j < prefix[1]
    gkeys = torch.where(valid, uniq[:nb], uniq[j % prefix[1].clamp_min(1)])
    assert torch.equal(va, valid)
    assert torch.equal(gk, gkeys)
    assert torch.equal(pc, pos) and pc.data_ptr() != pos.data_ptr()
    assert torch.equal(pr, torch.where(valid, gkeys, torch.full_like(gkeys, -1)))
