"""Shim of ``isaaclab.utils.assets.retrieve_file_path``: local paths only (no Nucleus offline)."""

import os


def retrieve_file_path(path: str, download_dir: str | None = None, force_download: bool = True) -> str:
    p = os.path.abspath(path)
    if not os.path.isfile(p):
        raise FileNotFoundError(f"Unable to find the file: {path}")
    return p
