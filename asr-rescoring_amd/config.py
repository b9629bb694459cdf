"""YAML config -> nested SimpleNamespace, mirroring util/config.py:3-15 + util/arg_parser.py:6-22.

The reference parses with ``ruamel.yaml`` (not installed here); PyYAML's ``safe_load`` reads
the same configs (plain mappings/scalars/lists).  Build-specific keys (``backend``,
``precision``, ``max_rows``, ``world_size``) are optional extras.
"""
from __future__ import annotations

import argparse
from types import SimpleNamespace

import yaml


def parse_config(config: dict) -> SimpleNamespace:
    out = SimpleNamespace()
    for k, v in config.items():
        setattr(out, k, parse_config(v) if isinstance(v, dict) else v)
    return out


def load_yaml(path: str) -> dict:
    with open(path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f) or {}


class ArgParser:
    """``--config <yaml>`` (util/arg_parser.py:6-22)."""

    def __init__(self) -> None:
        self.parser = argparse.ArgumentParser()
        self.parser.add_argument("--config", type=str, required=True, help="yaml configuration file path")

    def parse(self, argv=None) -> SimpleNamespace:
        args = self.parser.parse_args(argv)
        return parse_config(load_yaml(args.config))


def get(cfg: SimpleNamespace, dotted: str, default=None):
    cur = cfg
    for part in dotted.split("."):
        if not hasattr(cur, part):
            return default
        cur = getattr(cur, part)
    return cur
