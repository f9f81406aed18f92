from ._batchsampler import MegatronPretrainingRandomSampler, MegatronPretrainingSampler  # noqa: F401

__all__ = ["MegatronPretrainingSampler", "MegatronPretrainingRandomSampler"]
