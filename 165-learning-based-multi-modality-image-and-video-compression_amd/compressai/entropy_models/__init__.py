from .entropy_models import EntropyBottleneck, EntropyModel, GaussianConditional, seed_noise, set_noise_source

__all__ = ["EntropyModel", "EntropyBottleneck", "GaussianConditional", "set_noise_source", "seed_noise"]
