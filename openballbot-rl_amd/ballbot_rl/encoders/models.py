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
