"""Compact exact bf16 softcap (csrc/lens.hip CapC, used by decode_head): below ``lo`` the transformers chain
rbf(rbf(tanh(rbf(x / cap))) * cap) equals rbf(rbf(x * (1/cap)) * cap), from ``hi`` on it saturates, and only the
patterns in between need a table.  Checked here exhaustively for the caps Gemma-2 uses (final 30, attention 50):
every one of the 65536 bf16 inputs, through the same decomposition the kernel applies."""
import pytest
import torch

from taboo_brittleness_amd import ops
from taboo_brittleness_amd.ops import reference as ref

BF = torch.bfloat16


def _compact_values(x: torch.Tensor, tab: torch.Tensor, cap: float, lo: int, hi: int, sat: float) -> torch.Tensor:
    """CPU model of csrc/lens.hip capc1."""
    b = x.view(torch.int16).to(torch.int32) & 0xFFFF
    ab = b & 0x7FFF
    xf = x.float()
    a = ((xf * torch.tensor(1.0 / cap, dtype=torch.float32)).to(BF).float() * cap).to(BF).float()
    mag = torch.where(ab < hi, tab.float()[ab.clamp(max=32767)], torch.full_like(xf, sat))
    mag = torch.where(ab <= 0x7F80, mag, xf.abs())
    out = torch.where(ab < lo, a, torch.where((b & 0x8000) != 0, -mag, mag))
    return torch.where(ab > 0x7F80, xf, out)


@pytest.mark.parametrize("cap", [30.0, 50.0])
def test_compact_softcap_exhaustive(cap):
    bits = torch.arange(32768, dtype=torch.int32).to(torch.int16)
    tab = ref.softcap_bf16(bits.view(BF), cap).to(BF)
    split = ops.softcap_compact_split(tab, cap)
    assert split is not None
    lo, hi, sat = split
    assert 0 < lo < hi < 0x7F80 and hi - lo <= 2048 and sat == cap
    allx = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(BF)
    got = _compact_values(allx, tab, cap, lo, hi, sat)
    want = ref.softcap_bf16(allx, cap).float()
    same = (got == want) | (torch.isnan(got) & torch.isnan(want))
    assert same.all(), int((~same).sum())
