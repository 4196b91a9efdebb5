"""Non-executing loader for mmcv-style ``.py`` config files.

The reference's configs (projects/configs/**.py) are Python files made of
assignments of literals, dicts/lists/tuples, names defined earlier in the file,
``dict(...)`` calls and simple arithmetic / ``len()`` (e.g.
``num_classes=len(class_names)``, ``data_root + '/x.pkl'``).  mmcv's
``Config.fromfile`` executes them; this loader instead walks the AST and
evaluates only that whitelisted subset, so loading a config never runs code.
"""
import ast
import operator

__all__ = ["load_config", "loads_config", "ConfigError"]


class ConfigError(ValueError):
    pass


_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv,
           ast.FloorDiv: operator.floordiv, ast.Mod: operator.mod, ast.Pow: operator.pow}
_UNOPS = {ast.USub: operator.neg, ast.UAdd: operator.pos, ast.Not: operator.not_}
_FUNCS = {"dict": dict, "list": list, "tuple": tuple, "len": len, "range": lambda *a: list(range(*a)),
          "int": int, "float": float, "str": str, "min": min, "max": max, "sum": sum, "abs": abs}


def _eval(node, env):
    if isinstance(node, ast.Constant):
        return node.value
    if isinstance(node, ast.Name):
        if node.id in env:
            return env[node.id]
        if node.id in ("True", "False", "None"):
            return {"True": True, "False": False, "None": None}[node.id]
        raise ConfigError(f"undefined name {node.id!r} (line {node.lineno})")
    if isinstance(node, (ast.List, ast.Tuple, ast.Set)):
        items = [_eval(e, env) for e in node.elts]
        return tuple(items) if isinstance(node, ast.Tuple) else (set(items) if isinstance(node, ast.Set) else items)
    if isinstance(node, ast.Dict):
        return {_eval(k, env): _eval(v, env) for k, v in zip(node.keys, node.values)}
    if isinstance(node, ast.BinOp) and type(node.op) in _BINOPS:
        return _BINOPS[type(node.op)](_eval(node.left, env), _eval(node.right, env))
    if isinstance(node, ast.UnaryOp) and type(node.op) in _UNOPS:
        return _UNOPS[type(node.op)](_eval(node.operand, env))
    if isinstance(node, ast.Subscript):
        base = _eval(node.value, env)
        sl = node.slice
        if isinstance(sl, ast.Slice):
            lo = _eval(sl.lower, env) if sl.lower else None
            hi = _eval(sl.upper, env) if sl.upper else None
            st = _eval(sl.step, env) if sl.step else None
            return base[lo:hi:st]
        return base[_eval(sl, env)]
    if isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id in _FUNCS:
        args = [_eval(a, env) for a in node.args]
        kwargs = {}
        for k in node.keywords:
            if k.arg is None:          # dict(type=..., **img_norm_cfg)
                kwargs.update(_eval(k.value, env))
            else:
                kwargs[k.arg] = _eval(k.value, env)
        return _FUNCS[node.func.id](*args, **kwargs)
    if isinstance(node, ast.ListComp) or isinstance(node, ast.Lambda):
        raise ConfigError(f"unsupported construct at line {node.lineno}")
    raise ConfigError(f"unsupported expression {ast.dump(node)[:80]} (line {getattr(node, 'lineno', '?')})")


def loads_config(text):
    """Evaluate the assignment statements of a config file body -> dict."""
    tree = ast.parse(text)
    env = {}
    for stmt in tree.body:
        if isinstance(stmt, ast.Assign):
            val = _eval(stmt.value, env)
            for tgt in stmt.targets:
                if not isinstance(tgt, ast.Name):
                    raise ConfigError(f"only simple assignments are supported (line {stmt.lineno})")
                env[tgt.id] = val
        elif isinstance(stmt, ast.Expr) and isinstance(stmt.value, ast.Constant):
            continue   # docstring / bare string
        elif isinstance(stmt, (ast.Import, ast.ImportFrom)):
            raise ConfigError(f"imports are not allowed in configs (line {stmt.lineno})")
        else:
            raise ConfigError(f"unsupported statement {type(stmt).__name__} (line {stmt.lineno})")
    return env


def load_config(path):
    with open(path, "r") as f:
        return loads_config(f.read())
