"""Depth encoders (reference ballbot_rl/encoders)."""
from ballbot_rl.encoders.models import TinyAutoencoder, load_frozen_encoder, save_encoder
from ballbot_rl.encoders.pretrain import collect_depth_images, train_autoencoder

__all__ = ["TinyAutoencoder", "train_autoencoder", "collect_depth_images", "save_encoder", "load_frozen_encoder"]
