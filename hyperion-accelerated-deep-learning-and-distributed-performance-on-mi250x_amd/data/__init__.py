"""Data pipeline (reference L2: C11-C13): dataset wrappers, real-data adapters, synthetic sets, sampler."""
from .datasets import (  # noqa: F401
    CIFAR10TorchDataset,
    TensorPairDataset,
    WikiText2TorchDataset,
    load_cifar10_pt,
    load_wikitext2,
)
from .sampler import DistributedSampler  # noqa: F401
from .synthetic import SyntheticCIFAR10, SyntheticImageNet, SyntheticWikiText2  # noqa: F401
