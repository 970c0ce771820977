from .config import CfgNode, get_cfg, load_cfg  # noqa: F401
