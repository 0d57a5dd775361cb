"""Block layouts shared with the HIP library, parsed from ``csrc/dat_layout.h`` (single source of truth)."""

from __future__ import annotations

import os
import re

_HDR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "dat_layout.h")

_const: dict = {}
_func: dict = {}
with open(_HDR) as _f:
    for _line in _f:
        _m = re.match(r"#define\s+(DAT_\w+)\((\w+)\)\s+(.+?)\s*(//.*)?$", _line)
        if _m:
            _func[_m.group(1)] = (_m.group(2), _m.group(3))
            continue
        _m = re.match(r"#define\s+(DAT_\w+)\s+([-\w.()+* ]+?)\s*(//.*)?$", _line)
        if _m:
            _const[_m.group(1)] = _m.group(2)


def _eval(expr: str, env: dict):
    expr = re.sub(r"(DAT_\w+)\((\w+)\)", lambda m: str(fn(m.group(1), int(env[m.group(2)]) if m.group(2) in env else int(m.group(2)))), expr)
    expr = re.sub(r"\bDAT_\w+\b", lambda m: str(const(m.group(0))), expr)
    return eval(expr, {}, env)  # noqa: S307 -- header arithmetic only


def const(name: str):
    return _eval(_const[name], {})


def fn(name: str, n: int) -> int:
    arg, body = _func[name]
    return int(_eval(body, {arg: n}))


P = {k[len("DAT_P_"):]: const(k) for k in _const if k.startswith("DAT_P_")}
M = {k[len("DAT_M_"):]: const(k) for k in _const if k.startswith("DAT_M_")}
NENV = const("DAT_NENV")
GRAVITY = const("DAT_GRAVITY")


def param_size(n: int) -> int:
    return fn("DAT_PARAM_SIZE", n)


def state_size(n: int) -> int:
    return fn("DAT_STATE_SIZE", n)


def p_off(name: str, n: int) -> int:
    return fn("DAT_P_" + name, n)


def s_off(name: str, n: int) -> int:
    return fn("DAT_S_" + name, n)
