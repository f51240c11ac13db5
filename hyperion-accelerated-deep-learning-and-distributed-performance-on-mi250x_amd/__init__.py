"""Hyperion-MI355X: an MI355X-native (CDNA4 / gfx950) training and benchmarking framework.

Layer map:

* ``hyperion.utils``     device/arch probe, env knobs, seeding, hipEvent timers, memory stats, run manifest
* ``hyperion.config``    typed config (dataclasses) that is actually loaded (the reference's
                          ``Phase 1/default_config.json`` was dead)
* ``hyperion.data``      synthetic + real dataset adapters, distributed sampler
* ``hyperion.models``    ResNet-18/50, ViT-B/16, fallback CNN, custom Transformer, SimpleTransformerLM,
                          Llama (HF-key compatible), LoRA
* ``hyperion.ops``       autograd functions over hand-written gfx950 HIP kernels (``hyperion._C``)
* ``hyperion.parallel``  process-group setup, native RCCL communicator, DDP, FSDP
* ``hyperion.train``     AMP, activation checkpointing, trainers with reference-compatible APIs
* ``hyperion.bench``     hardware microbenchmarks, baseline step benchmark, scaling report
* ``hyperion.profiling`` roctx ranges, rocprofv3 wrappers
* ``hyperion.cli``       ``run_distributed`` / ``test_rccl`` / bench entry points
"""

__version__ = "0.1.0"

PACKAGE_DIR_NAME = "hyperion-accelerated-deep-learning-and-distributed-performance-on-mi250x_amd"
