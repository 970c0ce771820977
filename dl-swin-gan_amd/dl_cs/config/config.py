"""fvcore-free configuration (cfg = dl_cs/config/config.py:11-115, defaults.py:17-209).

Reads the same YAML keys as the reference (config_swin.yaml etc.) on top of the
same defaults; YAML tuples written as "(10, 15)" strings are parsed like the
reference's yacs literal_eval.  Merging an unknown key raises KeyError.
"""
import ast
import copy
import os

import yaml


class CfgNode(dict):
    """Attribute-access dict with freeze(), merge_from_file() and clone()."""

    def __init__(self, init=None):
        super().__init__()
        object.__setattr__(self, "_frozen", False)
        for k, v in (init or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) else v

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        if self._frozen:
            raise AttributeError(f"config is frozen; cannot set {name}")
        self[name] = value

    def freeze(self):
        object.__setattr__(self, "_frozen", True)
        for v in self.values():
            if isinstance(v, CfgNode):
                v.freeze()
        return self

    def clone(self):
        return CfgNode(copy.deepcopy(self.to_dict()))

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, CfgNode) else v) for k, v in self.items()}

    @staticmethod
    def _decode(v):
        if isinstance(v, str):
            try:
                return ast.literal_eval(v)
            except (ValueError, SyntaxError):
                return v
        return v

    def merge_from_dict(self, d, path=""):
        for k, v in d.items():
            if k not in self:
                raise KeyError(f"Non-existent config key: {path}{k}")
            if isinstance(self[k], CfgNode):
                if not isinstance(v, dict):
                    raise TypeError(f"{path}{k} must be a mapping")
                self[k].merge_from_dict(v, path + k + ".")
            else:
                v = self._decode(v)
                old = self[k]
                if isinstance(old, tuple) and isinstance(v, list):
                    v = tuple(v)
                self[k] = v

    def merge_from_file(self, filename):
        with open(filename) as f:
            d = yaml.safe_load(f) or {}
        self.merge_from_dict(d)


def get_cfg():
    from .defaults import _C
    return CfgNode(copy.deepcopy(_C))


def load_cfg(filename):
    """cfg:98-115"""
    if not os.path.isfile(filename):
        raise ValueError(f"Cannot find config file {filename}")
    cfg = get_cfg()
    cfg.merge_from_file(filename)
    cfg.freeze()
    if not cfg.OUTPUT_DIR:
        raise ValueError("OUTPUT_DIR not specified")
    return cfg
