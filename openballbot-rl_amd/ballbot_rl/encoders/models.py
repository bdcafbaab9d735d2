"""Depth-image autoencoder (reference ballbot_rl/encoders/models.py:6-54).

Same architecture: encoder = Conv(1->32, k3 s2 p1) BN LeakyReLU, Conv(32->32, k3 s2
p1) BN LeakyReLU, Flatten, Linear(32*H/4*W/4 -> 20), BatchNorm1d, Tanh (the
Extractor's rgbd branch, policies/mlp_policy.py:25-46); decoder mirrors it with
two ConvTranspose2d (output_padding 1) and a Sigmoid.  The pretrained encoder
becomes the policy's frozen rgbd extractor (train.py frozen_cnn).
"""
from __future__ import annotations

import torch
from torch import nn


class TinyAutoencoder(nn.Module):

    def __init__(self, H: int = 64, W: int = 64, in_c: int = 1, out_sz: int = 20):
        super().__init__()
        F1 = F2 = 32
        flat = F2 * (H // 4) * (W // 4)
        self.H, self.W, self.out_sz = H, W, out_sz
        self.encoder = nn.Sequential(
            nn.Conv2d(1, F1, kernel_size=3, stride=2, padding=1), nn.BatchNorm2d(F1), nn.LeakyReLU(),
            nn.Conv2d(F1, F2, kernel_size=3, stride=2, padding=1), nn.BatchNorm2d(F2), nn.LeakyReLU(),
            nn.Flatten(), nn.Linear(flat, out_sz), nn.BatchNorm1d(out_sz), nn.Tanh())
        self.decoder = nn.Sequential(
            nn.Linear(out_sz, flat), nn.BatchNorm1d(flat), nn.LeakyReLU(),
            nn.Unflatten(1, (F2, H // 4, W // 4)),
            nn.ConvTranspose2d(F2, F1, kernel_size=3, stride=2, padding=1, output_padding=1), nn.BatchNorm2d(F1),
            nn.LeakyReLU(),
            nn.ConvTranspose2d(F1, 1, kernel_size=3, stride=2, padding=1, output_padding=1), nn.Sigmoid())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.decoder(self.encoder(x))


def save_encoder(model: TinyAutoencoder, path: str) -> float:
    """Encoder weights as safetensors (+ JSON sidecar with H, W, out_sz and the
    reference's p_sum check value); returns p_sum.  The reference pickles the
    module with torch.save (training.py:68-73); safetensors executes nothing."""
    import json

    from safetensors.torch import save_file

    p_sum = float(sum(p.detach().abs().sum() for p in model.encoder.parameters() if p.requires_grad))
    save_file({k: v.detach().contiguous().cpu() for k, v in model.encoder.state_dict().items()}, path)
    with open(str(path) + ".json", "w") as f:
        json.dump({"H": model.H, "W": model.W, "out_sz": model.out_sz, "p_sum": p_sum}, f)
    return p_sum


def load_frozen_encoder(path: str, device="cpu") -> nn.Sequential:
    """The encoder of save_encoder(), in eval mode with requires_grad off, checked
    against its stored p_sum (the reference's corruption check, mlp_policy.py:108-125)."""
    import json

    from safetensors.torch import load_file

    with open(str(path) + ".json") as f:
        meta = json.load(f)
    enc = TinyAutoencoder(meta["H"], meta["W"], out_sz=meta["out_sz"]).encoder
    enc.load_state_dict(load_file(str(path), device=str(device)))
    p_sum = float(sum(p.detach().abs().sum() for p in enc.parameters()))
    if abs(p_sum - meta["p_sum"]) > 1e-5 * max(1.0, abs(meta["p_sum"])):
        raise ValueError(f"encoder parameter sum {p_sum} != stored {meta['p_sum']}: the file might be corrupted")
    for p in enc.parameters():
        p.requires_grad = False
    return enc.to(device).eval()


def fusable_encoder(enc: nn.Module) -> bool:
    """True when `enc` is the reference's frozen rgbd encoder layout (the encoder of
    TinyAutoencoder(64, 64): conv 1->32, BN, LeakyReLU(0.01), conv 32->32, BN,
    LeakyReLU, Flatten, Linear(8192 -> 20), BN1d, Tanh) with frozen fp32 weights
    and one BatchNorm momentum/eps, i.e. what bb_depth_encoder computes."""
    m = list(enc) if isinstance(enc, nn.Sequential) else []
    kinds = (nn.Conv2d, nn.BatchNorm2d, nn.LeakyReLU, nn.Conv2d, nn.BatchNorm2d, nn.LeakyReLU, nn.Flatten, nn.Linear,
             nn.BatchNorm1d, nn.Tanh)
    if len(m) != len(kinds) or any(type(x) is not k for x, k in zip(m, kinds)):
        return False
    c1, b1, a1, c2, b2, a2, _, fc, b3, _ = m
    conv_ok = all(c.bias is not None and c.kernel_size == (3, 3) and c.stride == (2, 2) and c.padding == (1, 1)
                  and c.dilation == (1, 1) and c.groups == 1 for c in (c1, c2))
    shapes_ok = (c1.in_channels, c1.out_channels, c2.in_channels, c2.out_channels) == (1, 32, 32, 32) and \
        (fc.in_features, fc.out_features) == (8192, 20) and fc.bias is not None
    bns = (b1, b2, b3)
    bn_ok = all(b.affine and b.track_running_stats and b.momentum is not None for b in bns) and \
        len({(float(b.momentum), float(b.eps)) for b in bns}) == 1 and (b1.num_features, b3.num_features) == (32, 20)
    act_ok = all(a.negative_slope == 0.01 for a in (a1, a2))
    frozen = all(not p.requires_grad for p in enc.parameters())
    dtypes = all(t.dtype == torch.float32 for t in list(enc.parameters()) + [b.running_mean for b in bns])
    return conv_ok and shapes_ok and bn_ok and act_ok and frozen and dtypes


def fused_encoder_forward(enc: nn.Sequential, x: torch.Tensor, index: "torch.Tensor | None" = None) -> torch.Tensor:
    """bb_depth_encoder on x [n, 1, 64, 64] (cuda, fp32; a channel slice of the
    [n, 2, 64, 64] camera tensor is fine): the frozen encoder's output [n, 20] with
    torch's BatchNorm semantics for enc.training (train: batch statistics and a
    running-statistics update; eval: running statistics).  No autograd graph.
    index (int64 [m], on the device): encode rows index[i] of x instead (a
    minibatch gathered inside the kernel); the output has m rows."""
    import ctypes as C

    from ballbot_gym import _native as N

    c1, b1, _, c2, b2, _, _, fc, b3, _ = list(enc)
    n = x.shape[0] if index is None else index.shape[0]
    if index is not None and (index.dtype != torch.int64 or not index.is_contiguous() or index.device != x.device):
        index = index.to(device=x.device, dtype=torch.int64).contiguous()
    if x.dim() != 4 or tuple(x.shape[1:]) != (1, 64, 64) or x.stride(3) != 1 or x.stride(2) != 64 \
            or x.stride(0) % 4 or x.data_ptr() % 16 or x.dtype != torch.float32:
        x = x.contiguous()
    ptr = lambda t: t.data_ptr()  # noqa: E731
    vals = [c1.weight, c1.bias, b1.weight, b1.bias, b1.running_mean, b1.running_var, b1.num_batches_tracked,
            c2.weight, c2.bias, b2.weight, b2.bias, b2.running_mean, b2.running_var, b2.num_batches_tracked,
            fc.weight, fc.bias, b3.weight, b3.bias, b3.running_mean, b3.running_var, b3.num_batches_tracked]
    p = N.EncoderParams(*[ptr(t.data if isinstance(t, nn.Parameter) else t) for t in vals])
    nbytes = C.c_int64()
    L = N.lib()
    N.check(L.bb_depth_encoder_workspace_bytes(int(n), C.byref(nbytes)), "bb_depth_encoder_workspace_bytes")
    ws = torch.empty(int(nbytes.value) // 4 + 4, device=x.device)
    out = torch.empty(n, 20, device=x.device)
    stream = C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    N.check(L.bb_depth_encoder(C.byref(p), C.c_void_p(x.data_ptr()), int(x.stride(0)),
                               None if index is None else C.c_void_p(index.data_ptr()), int(n), 64, 64,
                               int(bool(enc.training)), float(b1.momentum), float(b1.eps), C.c_void_p(out.data_ptr()),
                               20, C.c_void_p(ws.data_ptr()), int(nbytes.value), stream), "bb_depth_encoder")
    return out
