"""absl / ``tf.app.flags``-compatible flag system (reference: ``mnist_python_m.py:49-87, 323-324``).

    from tensorflow_distributed_amd import app
    flags = app.flags
    flags.DEFINE_string("data_dir", "/tmp/mnist-data", "...")
    FLAGS = flags.FLAGS
    app.run(main)

Accepts ``--name=value``, ``--name value``, ``--bool``/``--nobool`` and ``--bool=false`` forms,
like gflags. Unknown flags raise (as tf.app.run does), unless ``allow_unknown=True``.
"""
from __future__ import annotations

import sys
from typing import Any, Callable, Dict, List, Optional


class FlagError(ValueError):
    pass


class _Flag:
    def __init__(self, name: str, default: Any, help: str, parser: Callable[[str], Any], kind: str):
        self.name, self.default, self.help, self.parser, self.kind = name, default, help, parser, kind
        self.value = default
        self.present = False


def _parse_bool(s: str) -> bool:
    v = s.strip().lower()
    if v in ("1", "true", "t", "yes", "y"):
        return True
    if v in ("0", "false", "f", "no", "n"):
        return False
    raise FlagError(f"bad boolean value {s!r}")


class FlagValues:
    def __init__(self):
        object.__setattr__(self, "_flags", {})
        object.__setattr__(self, "_parsed", False)

    # -- definition --
    def _define(self, name, default, help, parser, kind):
        if name in self._flags:
            # re-definition with identical default is tolerated (scripts imported twice in tests)
            return
        self._flags[name] = _Flag(name, default, help, parser, kind)

    def __getattr__(self, name):
        flags = object.__getattribute__(self, "_flags")
        if name in flags:
            return flags[name].value
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in self._flags:
            self._flags[name].value = value
        else:
            raise AttributeError(f"unknown flag {name}")

    def __contains__(self, name):
        return name in self._flags

    def flag_values_dict(self) -> Dict[str, Any]:
        return {k: f.value for k, f in self._flags.items()}

    def reset(self):
        for f in self._flags.values():
            f.value, f.present = f.default, False
        object.__setattr__(self, "_parsed", False)

    def is_parsed(self) -> bool:
        return self._parsed

    # -- parsing --
    def parse(self, argv: List[str], allow_unknown: bool = False) -> List[str]:
        """Parse ``argv`` (argv[0] is the program). Returns the remaining positional args."""
        rest = [argv[0]] if argv else []
        i = 1
        while i < len(argv):
            a = argv[i]
            if a == "--":
                rest.extend(argv[i + 1:])
                break
            if not a.startswith("-") or a == "-":
                rest.append(a)
                i += 1
                continue
            body = a.lstrip("-")
            if "=" in body:
                name, val = body.split("=", 1)
            else:
                name, val = body, None
            name_u = name.replace("-", "_")
            f = self._flags.get(name_u)
            if f is None and val is None and name_u.startswith("no") and name_u[2:] in self._flags \
                    and self._flags[name_u[2:]].kind == "bool":
                f = self._flags[name_u[2:]]
                f.value, f.present = False, True
                i += 1
                continue
            if f is None:
                if allow_unknown:
                    rest.append(a)
                    i += 1
                    continue
                raise FlagError(f"Unknown command line flag '{name}'")
            if val is None:
                if f.kind == "bool":
                    f.value, f.present = True, True
                    i += 1
                    continue
                if i + 1 >= len(argv):
                    raise FlagError(f"flag --{name} needs a value")
                val = argv[i + 1]
                i += 1
            try:
                f.value = f.parser(val)
            except (TypeError, ValueError) as e:
                raise FlagError(f"bad value for --{name}: {val!r} ({e})")
            f.present = True
            i += 1
        object.__setattr__(self, "_parsed", True)
        return rest

    def __call__(self, argv: List[str], allow_unknown: bool = False) -> List[str]:
        return self.parse(argv, allow_unknown)

    def help_text(self) -> str:
        lines = []
        for f in self._flags.values():
            lines.append(f"  --{f.name}: {f.help} (default: {f.default!r})")
        return "\n".join(lines)


FLAGS = FlagValues()


def DEFINE_string(name: str, default: Optional[str], help: str, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, str, "string")


def DEFINE_integer(name: str, default: Optional[int], help: str, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, lambda s: int(s, 0) if isinstance(s, str) else int(s), "int")


def DEFINE_float(name: str, default: Optional[float], help: str, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, float, "float")


def DEFINE_boolean(name: str, default: Optional[bool], help: str, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, _parse_bool, "bool")


DEFINE_bool = DEFINE_boolean


def DEFINE_list(name: str, default, help: str, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, lambda s: [x for x in s.split(",") if x], "list")


def DEFINE_enum(name: str, default: str, choices, help: str, flag_values: FlagValues = FLAGS):
    choices = list(choices)

    def p(s):
        if s not in choices:
            raise ValueError(f"must be one of {choices}")
        return s

    flag_values._define(name, default, help, p, "enum")


def run(main: Optional[Callable] = None, argv: Optional[List[str]] = None):
    """``tf.app.run``: parse flags from sys.argv, call ``main(argv)``, exit with its return code."""
    argv = list(sys.argv if argv is None else argv)
    if "--help" in argv or "-h" in argv:
        print(f"usage: {argv[0]} [flags]\n{FLAGS.help_text()}")
        sys.exit(0)
    rest = FLAGS.parse(argv)
    main = main or sys.modules["__main__"].main
    sys.exit(main(rest))
