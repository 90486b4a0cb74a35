"""Shim of ``isaaclab.utils.io``: ``dump_yaml`` (dataclass configs as plain dicts) and ``dump_pickle``."""

from __future__ import annotations

import dataclasses
import os
import pickle


def _plain(obj):
    if dataclasses.is_dataclass(obj):
        return {f.name: _plain(getattr(obj, f.name)) for f in dataclasses.fields(obj)}
    if isinstance(obj, (list, tuple)):
        return [_plain(x) for x in obj]
    if isinstance(obj, dict):
        return {k: _plain(v) for k, v in obj.items()}
    return obj if isinstance(obj, (int, float, str, bool, type(None))) else repr(obj)


def dump_yaml(filename: str, data, sort_keys: bool = False) -> None:
    import yaml

    if not filename.endswith("yaml"):
        filename += ".yaml"
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    with open(filename, "w") as f:
        yaml.safe_dump(_plain(data), f, sort_keys=sort_keys)


def dump_pickle(filename: str, data) -> None:
    if not filename.endswith("pkl"):
        filename += ".pkl"
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    with open(filename, "wb") as f:
        pickle.dump(data, f)
