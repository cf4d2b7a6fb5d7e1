"""The reference's run configuration (config_file.json schema + parseit.py's command-line override
convention) read into the fusion model, optimizer and window shape this framework trains.

* load(path): the JSON file as the reference reads it (parseit.py:561-575);
* override(cfg, argv): parseit.py:293-345's rules — `--<top-level key>`, `--<model_params key>`
  (including every `opt__*` optimizer key), `--{train,val,test}_params__<key>` (the params dict
  or its loader_params); an unknown key raises as the reference does (ValueError /
  NotImplementedError); values are converted to the type the file holds (bools accept the
  reference's str2bool spellings);
* fusion_model(cfg): Two_transformers built as main.py:473-481 (vision_in_ft = 512: the R2D1 /
  ResNet18 features, main.py:469);
* sgd_kwargs(cfg): the `opt__*` SGD hyper-parameters (instantiator.py:30-36, the reference's
  optimizer for name_optimizer == "sgd");
* window(cfg): (batch_size, T) of a training batch: T = seq_length // subseq_length clips.
"""
from __future__ import annotations

import copy
import json
from typing import Dict, List, Sequence, Tuple

_PARAM_SETS = ("train_params", "val_params", "test_params")


def str2bool(v) -> bool:
    """parseit.py:53-63."""
    if isinstance(v, bool):
        return v
    s = str(v).lower()
    if s in ("yes", "true", "t", "y", "1"):
        return True
    if s in ("no", "false", "f", "n", "0"):
        return False
    raise ValueError(f"boolean value expected, got {v!r}")


def load(path: str) -> dict:
    with open(path, "r") as f:
        return json.load(f)


def _convert(old, val: str):
    if isinstance(old, bool):
        return str2bool(val)
    if isinstance(old, int):
        return int(val)
    if isinstance(old, float):
        return float(val)
    return val


def _pairs(argv: Sequence[str]) -> List[Tuple[str, str]]:
    out = []
    i = 0
    while i < len(argv):
        a = argv[i]
        if not a.startswith("--"):
            raise ValueError(f"expected --key, got {a!r}")
        if "=" in a:
            k, v = a[2:].split("=", 1)
            i += 1
        else:
            if i + 1 >= len(argv):
                raise ValueError(f"missing value for {a}")
            k, v = a[2:], argv[i + 1]
            i += 2
        out.append((k, v))
    return out


def override(cfg: dict, argv: Sequence[str]) -> dict:
    """A copy of cfg with parseit.py's `--key value` overrides applied."""
    cfg = copy.deepcopy(cfg)
    for k, v in _pairs(argv):
        if k in cfg and not isinstance(cfg[k], dict):
            cfg[k] = _convert(cfg[k], v)
        elif k in cfg.get("model_params", {}):
            cfg["model_params"][k] = _convert(cfg["model_params"][k], v)
        elif any(k.startswith(s + "__") for s in _PARAM_SETS):
            s, sub = k.split("__", 1)
            params = cfg[s]
            if sub in params and not isinstance(params[sub], dict):
                params[sub] = _convert(params[sub], v)
            elif sub in params.get("loader_params", {}):
                params["loader_params"][sub] = _convert(params["loader_params"][sub], v)
            else:
                raise NotImplementedError(f"Unknown key {k}")
        else:
            raise ValueError(f"Key {k} was not found in args. ... [NOT OK]")
    return cfg


def fusion_model(cfg: dict, vision_in_ft: int = 512, **kw):
    """main.py:473-481."""
    from models.two_transformers import Two_transformers
    mp = cfg["model_params"]
    return Two_transformers(v_dropout=float(mp["v_dropout"]), a_dropout=float(mp["a_dropout"]),
                            num_heads=int(mp["num_heads"]), num_layers=int(mp["num_layers"]),
                            joint_modalities=mp["joint_modalities"],
                            output_format=mp["output_format"], vision_in_ft=vision_in_ft, **kw)


def sgd_kwargs(cfg: dict) -> Dict[str, float]:
    mp = cfg["model_params"]
    name = str(mp.get("opt__name_optimizer", "sgd")).lower()
    if name != "sgd":
        raise NotImplementedError(f"opt__name_optimizer {name!r}: the fused optimizer is SGD")
    return dict(lr=float(mp["opt__lr"]), momentum=float(mp["opt__momentum"]),
                dampening=float(mp["opt__dampening"]),
                weight_decay=float(mp["opt__weight_decay"]),
                nesterov=str2bool(mp["opt__nesterov"]))


def window(cfg: dict, split: str = "train_params") -> Tuple[int, int]:
    p = cfg[split]
    return int(p["loader_params"]["batch_size"]), int(p["seq_length"]) // int(p["subseq_length"])
