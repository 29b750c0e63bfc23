"""CPU check of the test helper that decodes the kernels' ReLU bit image (tests/test_gpu_mlp.py
relu_bits): encode a random boolean [layers][rows][cols] pattern with the kernels' C-layout rule
(mlp_common.h mask_idx: bit i of lane (l32, h) of row tile rt, column tile t = row
rt*32 + (i & 3) + 8 (i >> 2) + 4 h, column t*32 + l32) and decode it back."""
import torch

from test_gpu_mlp import relu_bits


def _encode(B, hp):
    nh, M, _ = B.shape
    nt, n_rt = hp // 32, (M + 127) // 128 * 4
    w = torch.zeros(nh, n_rt, nt, 64, dtype=torch.int32)
    for rt in range(M // 32):
        for t in range(nt):
            for lane in range(64):
                l32, h = lane & 31, lane >> 5
                for i in range(16):
                    row = rt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h
                    w[:, rt, t, lane] |= B[:, row, t * 32 + l32].to(torch.int32) << i
    return w.to(torch.int16).flatten()


def test_relu_bits_roundtrip():
    g = torch.Generator().manual_seed(3)
    nh, hp, M, hidden = 2, 64, 96, 50
    B = torch.rand(nh, M, hp, generator=g) > 0.5
    got = relu_bits(_encode(B, hp), nh, hp, hidden, M)
    assert torch.equal(got, B[:, :, :hidden])
