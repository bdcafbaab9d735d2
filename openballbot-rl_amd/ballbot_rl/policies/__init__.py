"""Policy networks (reference ballbot_rl/policies/__init__.py:1-10): registers the
Extractor as policy plugin "mlp"."""
from ballbot_gym.core.registry import ComponentRegistry
from ballbot_rl.policies.mlp_policy import ActorCriticPolicy, Extractor, obs_spaces

if "mlp" not in ComponentRegistry.list_policies():
    ComponentRegistry.register_policy("mlp", Extractor)

__all__ = ["Extractor", "ActorCriticPolicy", "obs_spaces"]
