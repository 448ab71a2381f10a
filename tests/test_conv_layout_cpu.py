"""CPU checks of the host-side weight layouts the conv kernels consume.

* ``_s2_tap_perm``: the tap-permuted flipped weight of the one-launch stride-2
  3x3 data gradient (gemm.hip MultiGeo) holds, class after class, exactly the
  per-class weight subsets of the four-launch parity path
  (``_parity_weights``), so both launch forms read the same operands.
"""
import torch

from distributed_compute_pytorch_amd.ops.conv import _parity_weights, _s2_tap_perm


def test_s2_tap_perm_matches_parity_subsets():
    torch.manual_seed(0)
    cin, cout = 8, 12
    w = torch.randn(cout, cin, 3, 3)
    wd = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()  # [Cin][3][3][Cout], as the backward builds it
    perm = _s2_tap_perm(wd)
    assert perm.shape == (cin, 9, cout) and perm.is_contiguous()
    subs = _parity_weights(wd)
    off = 0
    for q, sub in enumerate(subs):
        n = sub.shape[1] * sub.shape[2]
        assert n == [1, 2, 2, 4][q]
        torch.testing.assert_close(perm[:, off:off + n, :], sub.reshape(cin, n, cout), rtol=0, atol=0)
        off += n
    assert off == 9
    # every tap exactly once
    assert torch.equal(perm.sort(dim=1).values, wd.reshape(cin, 9, cout).sort(dim=1).values)
