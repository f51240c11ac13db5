"""Reference-API trainers end to end on CPU (gloo world 2 and single process): CSV schemas,
checkpoint layout, resume, scaling report inputs."""
import csv
import glob
import os

import torch

from dist_utils import run_world


def _opts(**kw):
    from hyperion.train.distributed import RunOptions

    d = dict(dataset_size=64, max_steps_per_epoch=2, num_workers=0, log=lambda s: None)
    d.update(kw)
    return RunOptions(**d)


def _lm_ddp(rank, world, base):
    from hyperion.train.distributed import train_language_model_ddp

    return train_language_model_ddp(rank, world, epochs=2, base_dir=base, opts=_opts(), batch_size=4)


def test_language_ddp_world2_writes_reference_csv_and_checkpoint(tmp_path):
    res = run_world(_lm_ddp, 2, (str(tmp_path),))
    rid = res[0]["run_id"]
    assert rid.startswith("language_ddp_2gpus_")
    rows = list(csv.reader(open(tmp_path / "data" / "distributed" / f"{rid}_metrics.csv")))
    assert rows[0] == ["epoch", "loss", "duration", "gpus"] and len(rows) == 3 and rows[1][3] == "2"
    ck = torch.load(res[0]["checkpoint"], weights_only=True)
    assert "model_state_dict" in ck and "embed.weight" in ck["model_state_dict"]
    assert "optimizer_state_dict" in ck and ck["epoch"] == 2
    assert res[1]["checkpoint"] is None


def _cifar(rank, world, base):
    from hyperion.train.distributed import train_cifar_model_ddp

    return train_cifar_model_ddp(rank, world, epochs=1, base_dir=base, opts=_opts(), batch_size=4)


def test_cifar_ddp_world2_csv_has_accuracy(tmp_path):
    res = run_world(_cifar, 2, (str(tmp_path),))
    rid = res[0]["run_id"]
    rows = list(csv.reader(open(tmp_path / "data" / "distributed" / f"{rid}_metrics.csv")))
    assert rows[0] == ["epoch", "loss", "accuracy", "duration", "gpus"]
    assert 0.0 <= float(rows[1][2]) <= 100.0


def _fsdp(rank, world, base, resume):
    from hyperion.models.simple_lm import simple_lm_256
    from hyperion.train.distributed import train_language_model_fsdp

    small = lambda: simple_lm_256(vocab_size=50257, emb_dim=32, n_heads=2, ff_dim=64)  # noqa: E731
    return train_language_model_fsdp(rank, world, epochs=2, base_dir=base, opts=_opts(resume=resume), batch_size=4,
                                     model_fn=small, min_num_params=5000)


def test_fsdp_trainer_world2_full_checkpoint_and_resume(tmp_path):
    res = run_world(_fsdp, 2, (str(tmp_path), None))
    path = res[0]["checkpoint"]
    ck = torch.load(path, weights_only=True)
    assert "tr.layers.0.linear1.weight" in ck["model_state_dict"]  # original keys, full tensors
    assert ck["model_state_dict"]["tr.layers.0.linear1.weight"].shape == (64, 32)
    assert os.path.exists(path.replace(".pt", "_optim_rank1.pt"))
    res2 = run_world(_fsdp, 2, (str(tmp_path), path))  # resume at epoch 2 of 2: no more epochs
    assert res2[0]["history"] == []


def _llama(rank, world, base, lora):
    from hyperion.models.llama import LlamaConfig
    from hyperion.train.distributed import train_llama_fsdp

    return train_llama_fsdp(rank, world, epochs=1, base_dir=base, lora=lora, batch_size=2, progress_every=0,
                            opts=_opts(), config=LlamaConfig.tiny())


def test_llama_lora_under_fsdp_saves_peft_adapter(tmp_path):
    res = run_world(_llama, 2, (str(tmp_path), True))
    d = res[0]["checkpoint"]
    assert os.path.exists(os.path.join(d, "adapter_model.safetensors"))
    rows = list(csv.reader(open(glob.glob(str(tmp_path / "data" / "distributed" / "llama_2gpus_*_metrics.csv"))[0])))
    assert rows[0] == ["epoch", "loss", "duration_s", "gpus", "mode"] and rows[1][4] == "lora_fp32"


def test_llama_full_fsdp_single_process(tmp_path):
    from hyperion.models.llama import LlamaConfig
    from hyperion.train.distributed import train_llama_fsdp

    r = train_llama_fsdp(0, 1, epochs=1, base_dir=str(tmp_path), lora=False, batch_size=2, progress_every=0,
                         opts=_opts(), config=LlamaConfig.tiny())
    assert r["mode"] == "fsdp_fp32" and r["history"][0]["steps"] == 2


def _final_params(base, **kw):
    from hyperion.train.distributed import train_language_model_ddp

    r = train_language_model_ddp(0, 1, epochs=2, base_dir=base, opts=_opts(**kw), batch_size=4)
    ck = torch.load(r["checkpoint"], weights_only=True)
    return r, ck


def test_restart_auto_resume_replays_the_lost_steps_bit_exact(tmp_path, monkeypatch):
    """Checkpoint every step; an injected failure at global step 3 kills the first run; a second
    run with resume='auto' continues from the latest checkpoint (epoch 1, batch 1) and ends with
    exactly the weights and optimizer state of an uninterrupted run (data position + RNG restored)."""
    from hyperion.utils.fault import InjectedFault

    ref_dir, run_dir = tmp_path / "ref", tmp_path / "run"
    _, ref = _final_params(str(ref_dir), ckpt_every=1)
    monkeypatch.setenv("HYPERION_FAULT", "0:3:raise")
    monkeypatch.setenv("HYPERION_FAULT_MARKER", str(tmp_path / "fault.marker"))
    import pytest

    with pytest.raises(InjectedFault):
        _final_params(str(run_dir), ckpt_every=1)
    latest = torch.load(run_dir / "data" / "distributed" / "language_ddp_latest.pt", weights_only=True)
    assert latest["step"] == 3 and latest["epoch"] == 1 and latest["step_in_epoch"] == 1
    r, got = _final_params(str(run_dir), ckpt_every=1, resume="auto")  # marker set: no second fault
    assert [h["steps"] for h in r["history"]] == [1]  # only the remaining step of epoch 2 re-ran
    for k, v in ref["model_state_dict"].items():
        assert torch.equal(v, got["model_state_dict"][k]), k
    rows = list(csv.reader(open(run_dir / "data" / "distributed" / f"{r['run_id']}_metrics.csv")))
    assert rows[0] == ["epoch", "loss", "duration", "gpus"] and [row[0] for row in rows[1:]] == ["1", "2"]


def test_cli_max_restarts_recovers_single_process(tmp_path, monkeypatch):
    from hyperion.cli.run_distributed import main

    monkeypatch.setenv("HYPERION_FAULT", "0:2:raise")
    monkeypatch.setenv("HYPERION_FAULT_MARKER", str(tmp_path / "m"))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    rc = main(["--model", "language_ddp", "--epochs", "2", "--max_steps", "2", "--dataset_size", "64", "--base_dir",
               str(tmp_path), "--ckpt_every", "1", "--max_restarts", "1"])
    assert rc == 0 and (tmp_path / "m").exists()
    assert (tmp_path / "data" / "distributed" / "language_ddp_latest.pt").exists()


def test_cli_restart_argv_rewrites_model_and_resume():
    from hyperion.cli.run_distributed import _child_argv

    a = ["--model", "all", "--epochs", "2", "--max_restarts", "3", "--resume=ckpt.pt", "--seed", "1"]
    assert _child_argv(a, "cifar", None) == ["--epochs", "2", "--seed", "1", "--model", "cifar"]
    assert _child_argv(a, "cifar", "auto")[-2:] == ["--resume", "auto"]


def _gpt2_fsdp(rank, world, base):
    from hyperion.train.distributed import train_language_model_fsdp
    from hyperion.models.simple_lm import gpt2_small_lm

    tiny = lambda: gpt2_small_lm(vocab_size=50257, emb_dim=32, n_heads=2, n_layers=2, ff_dim=64)  # noqa: E731
    return train_language_model_fsdp(rank, world, epochs=1, base_dir=base, opts=_opts(), batch_size=4, model_fn=tiny,
                                     wrap="layer", run_name="gpt2_fsdp")


def test_gpt2_fsdp_layer_units_world2(tmp_path):
    res = run_world(_gpt2_fsdp, 2, (str(tmp_path),))
    assert res[0]["run_id"].startswith("gpt2_fsdp_2gpus_")
    rows = list(csv.reader(open(tmp_path / "data" / "distributed" / f"{res[0]['run_id']}_metrics.csv")))
    assert rows[0] == ["epoch", "loss", "duration", "gpus"] and len(rows) == 2
