from .entropy_models import EntropyBottleneck, EntropyModel, GaussianConditional, set_noise_source

__all__ = ["EntropyModel", "EntropyBottleneck", "GaussianConditional", "set_noise_source"]
