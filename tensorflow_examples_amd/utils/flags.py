"""absl/tf.app.flags-compatible flag system (absl is not installed here).

Reproduces the reference's usage (R/distributed/distributed.py:24-32):

* ``DEFINE_string / DEFINE_integer / DEFINE_float / DEFINE_boolean (DEFINE_bool) / DEFINE_list``
  with ``(name, default, help)``;
* ``FLAGS.<name>`` triggers a LAZY parse of ``sys.argv`` on first access, known flags only
  (TF1's ``tf.flags`` wrapper parses with ``known_only=True`` when a flag is read before
  ``tf.app.run``; the reference never calls ``tf.app.run`` and first reads flags at :37);
* ``--name=value`` and ``--name value`` forms, ``--flag`` / ``--noflag`` for booleans,
  ``-name`` single-dash accepted like absl;
* unknown flags are left in ``FLAGS.unparsed_args``; explicit ``FLAGS(argv)`` parses fully.
"""
from __future__ import annotations

import sys
from typing import Any, Callable, Dict, List, Optional


class FlagsError(ValueError):
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
    raise FlagsError(f"invalid boolean value {s!r}")


class FlagValues:
    def __init__(self):
        object.__setattr__(self, "_flags", {})
        object.__setattr__(self, "_parsed", False)
        object.__setattr__(self, "unparsed_args", [])

    # ---------------------------------------------------------------- definition
    def _define(self, name, default, help, parser, kind):
        if name in self._flags:
            raise FlagsError(f"flag --{name} defined twice")
        self._flags[name] = _Flag(name, default, help, parser, kind)

    # ---------------------------------------------------------------- parsing
    def __call__(self, argv: Optional[List[str]] = None, known_only: bool = False) -> List[str]:
        argv = list(sys.argv if argv is None else argv)
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
            name, eq, val = body.partition("=")
            f = self._flags.get(name)
            if f is None and name.startswith("no") and not eq:
                g = self._flags.get(name[2:])
                if g is not None and g.kind == "bool":
                    g.value, g.present = False, True
                    i += 1
                    continue
            if f is None:
                if known_only:
                    rest.append(a)
                    i += 1
                    continue
                raise FlagsError(f"Unknown command line flag '{name}'")
            if f.kind == "bool" and not eq:
                f.value, f.present = True, True
                i += 1
                continue
            if not eq:
                if i + 1 >= len(argv):
                    raise FlagsError(f"flag --{name} needs a value")
                val = argv[i + 1]
                i += 1
            try:
                f.value = f.parser(val)
            except (ValueError, TypeError) as e:
                raise FlagsError(f"flag --{name}={val!r}: {e}") from None
            f.present = True
            i += 1
        object.__setattr__(self, "_parsed", True)
        object.__setattr__(self, "unparsed_args", rest)
        return rest

    def is_parsed(self) -> bool:
        return self._parsed

    def mark_as_parsed(self):
        object.__setattr__(self, "_parsed", True)

    def unparse_flags(self):
        for f in self._flags.values():
            f.value, f.present = f.default, False
        object.__setattr__(self, "_parsed", False)

    # ---------------------------------------------------------------- access
    def __getattr__(self, name):
        flags = object.__getattribute__(self, "_flags")
        if name not in flags:
            raise AttributeError(name)
        if not object.__getattribute__(self, "_parsed"):
            self(sys.argv, known_only=True)  # TF1 lazy parse
        return flags[name].value

    def __setattr__(self, name, value):
        if name in self._flags:
            self._flags[name].value = value
            self._flags[name].present = True
        else:
            raise AttributeError(f"unknown flag {name}")

    def __contains__(self, name):
        return name in self._flags

    def flag_values_dict(self) -> Dict[str, Any]:
        if not self._parsed:
            self(sys.argv, known_only=True)
        return {k: f.value for k, f in self._flags.items()}

    def __getitem__(self, name):
        return self._flags[name]

    def help_text(self) -> str:
        return "\n".join(f"  --{f.name}: {f.help}\n    (default: {f.default!r})" for f in self._flags.values())


FLAGS = FlagValues()


def DEFINE_string(name, default, help, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, str, "string")


def DEFINE_integer(name, default, help, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, int, "int")


def DEFINE_float(name, default, help, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, float, "float")


def DEFINE_boolean(name, default, help, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, _parse_bool, "bool")


DEFINE_bool = DEFINE_boolean


def DEFINE_list(name, default, help, flag_values: FlagValues = FLAGS):
    flag_values._define(name, default, help, lambda s: [x for x in s.split(",") if x], "list")
