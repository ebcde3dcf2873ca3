"""Config helpers (reference core/util.py:31-40)."""
from __future__ import annotations

from typing import Dict


def deep_dict_merge(dest: Dict, source: Dict) -> Dict:
    """Recursively merge ``source`` into ``dest`` in place and return ``dest``: nested dicts
    are merged key by key, every other value overwrites (reference util.py:31-40)."""
    for key, value in source.items():
        if isinstance(value, dict):
            deep_dict_merge(dest.setdefault(key, {}), value)
        else:
            dest[key] = value
    return dest
