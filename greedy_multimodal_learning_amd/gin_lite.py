"""A dependency-free subset of gin-config, enough for the reference's configs.

The reference wires everything through gin (`@gin.configurable` on
MMTM_MVCNN, train, eval_, training_loop, callbacks ...; CLI in
src/utils.py:58-68).  gin is not installed here, so this module accepts the
reference's five `.gin` files unchanged: `Scope.param = <python literal>`
lines, `#` comments, multi-line list literals, and `a=1#b=2`-style binding
strings.  Bound values fill the parameters a caller does not pass explicitly.
If the real `gin` package is importable, `configurable` defers to it.
"""
import ast
import functools
import inspect

_CONFIG = {}            # {(scope, name): {param: value}} like gin.config._CONFIG
_REGISTRY = {}


def _key(name):
    return ("", name)


def configurable(obj=None, *, name=None):
    if obj is None:
        return lambda o: configurable(o, name=name)
    reg_name = name or obj.__name__
    _REGISTRY[reg_name] = obj
    if inspect.isclass(obj):
        init = obj.__init__
        sig = inspect.signature(init)

        @functools.wraps(init)
        def wrapped_init(self, *args, **kwargs):
            kwargs = _fill(reg_name, sig, args, kwargs, skip_self=True)
            init(self, *args, **kwargs)
        obj.__init__ = wrapped_init
        return obj
    sig = inspect.signature(obj)

    @functools.wraps(obj)
    def wrapped(*args, **kwargs):
        return obj(*args, **_fill(reg_name, sig, args, kwargs))
    _REGISTRY[reg_name] = wrapped
    return wrapped


def _fill(reg_name, sig, args, kwargs, skip_self=False):
    bound = _CONFIG.get(_key(reg_name))
    if not bound:
        return kwargs
    params = list(sig.parameters)
    if skip_self:
        params = params[1:]
    positional = set(params[:len(args)])
    out = dict(kwargs)
    for k, v in bound.items():
        if k in positional or k in out:
            continue
        if k not in sig.parameters and not any(
                p.kind == p.VAR_KEYWORD for p in sig.parameters.values()):
            raise ValueError(f"gin_lite: {reg_name} has no parameter {k!r}")
        out[k] = v
    return out


def _statements(text):
    """Yield complete `lhs = rhs` statements (joins multi-line bracketed values)."""
    buf, depth = "", 0
    for raw in text.splitlines():
        line = raw.split("#", 1)[0] if depth == 0 else raw
        if "#" in line and depth:
            line = line.split("#", 1)[0]
        if not line.strip() and depth == 0:
            continue
        buf += line + "\n"
        depth += sum(line.count(c) for c in "([{") - sum(line.count(c) for c in ")]}")
        if depth <= 0:
            if buf.strip():
                yield buf.strip()
            buf, depth = "", 0
    if buf.strip():
        yield buf.strip()


def parse_config(text):
    for stmt in _statements(text):
        if stmt.startswith(("import ", "include ")):
            continue
        lhs, rhs = stmt.split("=", 1)
        lhs = lhs.strip()
        scope_name, param = lhs.rsplit(".", 1)
        scope_name = scope_name.split("/")[-1]
        val = rhs.strip()
        try:
            value = ast.literal_eval(val)
        except (ValueError, SyntaxError):
            if val.startswith("@"):
                value = val
            else:
                raise ValueError(f"gin_lite: cannot parse value of {lhs}: {val!r}")
        _CONFIG.setdefault(_key(scope_name), {})[param] = value


def parse_config_files_and_bindings(config_files, bindings):
    for f in config_files or []:
        if f:
            with open(f) as fh:
                parse_config(fh.read())
    if isinstance(bindings, (list, tuple)):
        bindings = "\n".join(bindings)
    if bindings:
        parse_config(bindings.replace("#", "\n") if "\n" not in bindings else bindings)


def query(name, param, default=None):
    return _CONFIG.get(_key(name), {}).get(param, default)


def clear_config():
    _CONFIG.clear()


def config_str():
    lines = []
    for (_, n), kv in sorted(_CONFIG.items()):
        for k, v in kv.items():
            lines.append(f"{n}.{k} = {v!r}")
    return "\n".join(lines)
