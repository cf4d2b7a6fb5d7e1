"""The config_file.json schema launcher (jmt/config.py): parseit.py's override convention and the
model / optimizer / window it yields (main.py:473-481, instantiator.py:30-36), CPU only."""
import os

import pytest

from jmt import config as C

REF_CFG = "/root/reference/config_file.json"


def _schema():
    """The keys of the shipped schema that the fusion path reads (config_file.json layout)."""
    loader = {"batch_size": 64, "shuffle": False, "num_workers": 4, "pin_memory": False}
    split = lambda: {"seq_length": 512, "subseq_length": 32, "stride": 1, "dilation": 4,
                     "loader_params": dict(loader)}
    return {"cudaid": "0", "verbose": "True", "SEED": 0, "goal": "TRAINING",
            "train_params": dict(split(), take_n_videos=-1), "val_params": split(),
            "test_params": split(),
            "model_params": {"output_format": "FC", "joint_modalities": "TRANSFORMER",
                             "num_layers": 1, "num_heads": 1, "v_dropout": 0.0, "a_dropout": 0.0,
                             "opt__name_optimizer": "sgd", "opt__lr": 1e-4, "opt__momentum": 0.9,
                             "opt__dampening": 0.0, "opt__weight_decay": 1e-4,
                             "opt__nesterov": "True", "max_epochs": 20}}


def test_defaults_window_and_sgd():
    cfg = _schema()
    assert C.window(cfg) == (64, 16)                     # 512 / 32 clips per window
    assert C.sgd_kwargs(cfg) == dict(lr=1e-4, momentum=0.9, dampening=0.0, weight_decay=1e-4,
                                     nesterov=True)


def test_overrides_follow_parseit():
    cfg = _schema()
    out = C.override(cfg, ["--num_heads", "2", "--opt__lr", "1e-3", "--opt__nesterov", "False",
                           "--train_params__batch_size", "32", "--train_params__seq_length=256",
                           "--output_format", "SELF_ATTEN", "--SEED", "7",
                           "--val_params__num_workers", "2"])
    assert cfg["model_params"]["num_heads"] == 1                         # input untouched
    mp = out["model_params"]
    assert mp["num_heads"] == 2 and isinstance(mp["num_heads"], int)
    assert mp["opt__lr"] == 1e-3 and mp["output_format"] == "SELF_ATTEN"
    assert C.sgd_kwargs(out)["nesterov"] is False
    assert C.window(out) == (32, 8)
    assert out["SEED"] == 7 and out["val_params"]["loader_params"]["num_workers"] == 2
    with pytest.raises(ValueError):
        C.override(cfg, ["--no_such_key", "1"])
    with pytest.raises(NotImplementedError):
        C.override(cfg, ["--train_params__no_such_key", "1"])


def test_fusion_model_from_config():
    import inspect
    from models.two_transformers import Two_transformers
    cfg = C.override(_schema(), ["--num_heads", "2", "--joint_modalities", "NONE"])
    m = C.fusion_model(cfg)
    assert isinstance(m, Two_transformers)
    assert (m.num_heads, m.num_layers, m.joint_modalities, m.output_format, m.vision_in_ft) == \
        (2, 1, "NONE", "FC", 512)


@pytest.mark.skipif(not os.path.exists(REF_CFG), reason="reference checkout absent")
def test_reads_the_reference_config_file():
    cfg = C.load(REF_CFG)
    assert C.window(cfg) == (64, 16)
    kw = C.sgd_kwargs(cfg)
    assert kw["nesterov"] is True and kw["lr"] == 1e-4
    m = C.fusion_model(cfg)
    assert (m.joint_modalities, m.output_format) == ("TRANSFORMER", "FC")
