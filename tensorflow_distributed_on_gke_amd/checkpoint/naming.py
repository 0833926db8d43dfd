"""Collision-free naming of snapshot folders.

Same semantics as the reference's helpers
(reference: distributed_training_transformer/checkpoint.py:134-170
`new_directory_name`, `unique_name`): try the bare name, then `_2`, `_3`, ...
(`number_first_name=True` starts at `_1`).
"""
from __future__ import annotations

from pathlib import Path
from typing import Callable


def unique_name(prefix: str, check_name_exists: Callable[[str], bool], suffix: str = "",
                index_separator: str = "_", number_first_name: bool = False) -> str:
    index = 1
    while True:
        if index == 1 and not number_first_name:
            name = prefix + suffix
        else:
            name = f"{prefix}{index_separator}{index}{suffix}"
        if check_name_exists(name):
            index += 1
        else:
            return name


def new_directory_name(base_name: str) -> str:
    return unique_name(base_name, lambda name: Path(name).exists())
