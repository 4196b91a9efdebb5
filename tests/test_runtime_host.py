"""Host-side numerics-policy checks (no GPU): the f16 operand range guard of
the 'ref' and 'fp16' policies (runtime.check_f16_range)."""
import pytest
import torch

from projects.mmdet3d_plugin.runtime import F16_MAX, PRECISIONS, check_f16_range


@pytest.mark.parametrize("prec", ["ref", "fp16"])
def test_f16_range_guard_raises_for_out_of_range_inputs(prec):
    p = PRECISIONS[prec]
    ok = torch.full((4, 8), F16_MAX)
    check_f16_range(p, [ok, None, torch.empty(0)])
    for bad in (F16_MAX * 1.01, float("inf"), float("nan")):
        x = ok.clone()
        x[2, 3] = -bad
        with pytest.raises(ValueError, match="exact"):
            check_f16_range(p, [ok, x])


@pytest.mark.parametrize("prec", ["exact", "bf16"])
def test_f16_range_guard_is_off_for_wide_policies(prec):
    check_f16_range(PRECISIONS[prec], [torch.full((2, 2), 1e30)])
