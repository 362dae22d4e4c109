"""Hydra/OmegaConf-compatible config composition (hydra-core / omegaconf are not installable
offline). Implements what the reference's configs use:

* the four custom resolvers of utils/hydra_cfg/hydra_utils.py:36-41 — ``eq``, ``contains``,
  ``if``, ``resolve_default``;
* absolute ``${a.b}`` and relative ``${.x}`` / ``${..x}`` / ``${...x}`` interpolation
  (OmegaConf semantics: one dot = the node holding the key, each extra dot one level up);
* the defaults list of cfg/config.yaml (``task`` and ``train: ${task}PPO`` groups);
* command-line style overrides ``task=Humanoid num_envs=64 task.env.episodeLength=100``
  (README.md:157-173).
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, List, Optional, Sequence

import yaml

CFG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "cfg")


def _as_str(x: Any) -> str:
    return "" if x is None else str(x)


RESOLVERS = {
    "eq": lambda x, y: _as_str(x).lower() == _as_str(y).lower(),
    "contains": lambda x, y: _as_str(x).lower() in _as_str(y).lower(),
    "if": lambda pred, a, b: a if pred else b,
    "resolve_default": lambda default, arg: default if arg == "" or arg is None else arg,
}


class InterpolationError(KeyError):
    pass


def _scalar(tok: str) -> Any:
    t = tok.strip()
    if len(t) >= 2 and t[0] == t[-1] and t[0] in "\"'":
        return t[1:-1]
    try:
        v = yaml.safe_load(t)
    except yaml.YAMLError:
        return t
    return "" if v is None and t == "" else v


def _split_args(s: str) -> List[str]:
    out, depth, cur, quote = [], 0, [], None
    for ch in s:
        if quote:
            cur.append(ch)
            if ch == quote:
                quote = None
            continue
        if ch in "\"'":
            quote = ch
        elif ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
        elif ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
            continue
        cur.append(ch)
    out.append("".join(cur))
    return out


class _Resolver:
    def __init__(self, root: Dict[str, Any]):
        self.root = root

    def lookup(self, path: str, node_path: List[str]) -> Any:
        if path.startswith("."):
            n = len(path) - len(path.lstrip("."))
            base = node_path[: len(node_path) - (n - 1)] if n - 1 <= len(node_path) else None
            if base is None:
                raise InterpolationError(path)
            keys = base + [k for k in path[n:].split(".") if k]
        else:
            keys = [k for k in path.split(".") if k]
        cur: Any = self.root
        for i, k in enumerate(keys):
            if not isinstance(cur, dict) or k not in cur:
                raise InterpolationError(f"${{{path}}} (at {'.'.join(node_path)})")
            cur = cur[k]
            if isinstance(cur, str) and "${" in cur:
                cur = self.value(cur, keys[: i])
        return cur

    def expr(self, body: str, node_path: List[str]) -> Any:
        name, sep, rest = body.partition(":")
        if sep and name in RESOLVERS:
            args = [self.value(a.strip(), node_path) if "${" in a else _scalar(a)
                    for a in _split_args(rest)]
            return RESOLVERS[name](*args)
        return self.lookup(body.strip(), node_path)

    def value(self, s: str, node_path: List[str]) -> Any:
        """Resolve every ${...} in s; a string that is exactly one interpolation keeps the
        referenced value's type."""
        out: List[Any] = []
        i = 0
        while i < len(s):
            j = s.find("${", i)
            if j < 0:
                out.append(s[i:])
                break
            out.append(s[i:j])
            depth, k = 0, j
            while k < len(s):
                if s[k] == "{":
                    depth += 1
                elif s[k] == "}":
                    depth -= 1
                    if depth == 0:
                        break
                k += 1
            out.append(self.expr(s[j + 2:k], node_path))
            i = k + 1
        parts = [p for p in out if not (isinstance(p, str) and p == "")]
        if len(parts) == 1 and not isinstance(parts[0], str):
            return parts[0]
        if len(out) == 1:
            return out[0]
        return "".join(_as_str(p) if not isinstance(p, bool) else str(p) for p in out)

    def resolve_tree(self, node: Any, path: List[str]) -> Any:
        if isinstance(node, dict):
            return {k: self.resolve_tree(v, path + [k]) for k, v in node.items()}
        if isinstance(node, list):
            return [self.resolve_tree(v, path) for v in node]
        if isinstance(node, str) and "${" in node:
            return self.value(node, path[:-1])
        return node


def resolve(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """Return a copy of cfg with every interpolation resolved."""
    return _Resolver(cfg).resolve_tree(copy.deepcopy(cfg), [])


def _load(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def _set_dotted(cfg: Dict[str, Any], key: str, value: Any) -> None:
    keys = key.split(".")
    cur = cfg
    for k in keys[:-1]:
        cur = cur.setdefault(k, {})
    cur[keys[-1]] = value


def compose(overrides: Optional[Sequence[str]] = None, cfg_dir: str = CFG_DIR) -> Dict[str, Any]:
    """Compose cfg/config.yaml + cfg/task/<task>.yaml + cfg/train/<train>.yaml, apply
    overrides, resolve interpolations — the equivalent of @hydra.main in
    scripts/rlgames_train.py:87-134."""
    overrides = list(overrides or [])
    top = _load(os.path.join(cfg_dir, "config.yaml"))
    defaults = top.pop("defaults", [])
    groups: Dict[str, str] = {}
    for d in defaults:
        if isinstance(d, dict):
            groups.update({k: v for k, v in d.items() if k in ("task", "train")})
    rest = []
    for ov in overrides:
        k, _, v = ov.partition("=")
        k = k.lstrip("+")          # Hydra's "+key=value" (append a key absent from the YAML)
        if k in ("task", "train"):
            groups[k] = v
        else:
            rest.append((k, _scalar(v)))
    task_name = groups.get("task", "Cartpole")
    train_name = groups.get("train", "${task}PPO").replace("${task}", task_name)
    top["task"] = _load(os.path.join(cfg_dir, "task", f"{task_name}.yaml"))
    train_path = os.path.join(cfg_dir, "train", f"{train_name}.yaml")
    top["train"] = _load(train_path) if os.path.exists(train_path) else {}
    for k, v in rest:
        _set_dotted(top, k, v)
    return resolve(top)
