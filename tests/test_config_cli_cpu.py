"""Config loading (the reference's dead config now has a reader) and CLI parsing."""
import json

import pytest

from hyperion.config import HyperionConfig, from_dict, load_config

REF_CFG = "/root/reference/Phase 1/default_config.json"


def test_reference_dead_config_loads(tmp_path):
    import os

    if not os.path.exists(REF_CFG):
        pytest.skip("reference config not present")
    cfg = load_config(REF_CFG)
    assert cfg.hardware.gpu_type == "MI250X" and cfg.optimization.compile_mode == "reduce-overhead"
    assert cfg.benchmarking.batch_sizes[-1] == 128 and cfg.distributed.backend == "nccl"


def test_unknown_keys_rejected():
    with pytest.raises(ValueError):
        from_dict({"optimization": {"nonexistent": 1}})


def test_yaml_roundtrip_and_apply(tmp_path):
    import yaml

    from hyperion.cli.run_distributed import build_parser
    from hyperion.config import apply_to_args

    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump({"training": {"epochs": 2, "max_steps": 3}, "optimization": {"kernels": "torch"}}))
    cfg = load_config(str(p))
    args = build_parser().parse_args(["--model", "cifar", "--epochs", "7"])
    apply_to_args(cfg, args)
    assert args.epochs == 7  # explicit flag wins
    assert args.max_steps == 3 and args.kernels == "torch"


def test_default_config_file_matches_dataclass():
    d = json.load(open("configs/default_mi355x.json"))
    assert from_dict(d) == HyperionConfig()


def test_run_distributed_single_process_cifar(tmp_path):
    from hyperion.cli.run_distributed import main

    rc = main(["--model", "cifar", "--epochs", "1", "--base_dir", str(tmp_path), "--max_steps", "1",
               "--dataset_size", "16", "--no_save"])
    assert rc == 0
    assert list((tmp_path / "data" / "distributed").glob("cifar_ddp_1gpus_*_metrics.csv"))
