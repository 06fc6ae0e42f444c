"""Commons-CLI compatible option-string parser.

Hivemall functions take their hyper-parameters as the last constant string argument,
e.g. ``train_classifier(features, label, '-loss logloss -opt adagrad -iters 20')``.
Upstream parses it with Apache Commons CLI's ``BasicParser`` inside
``UDTFWithOptions.parseOptions`` / ``UDFWithOptions`` (reference:
core/src/main/java/hivemall/UDTFWithOptions.java).  The observable rules,
reproduced here:

* the string is split on whitespace;
* an option is spelled ``-name`` or ``--name`` and matches either its short or its long
  name (Commons CLI strips leading hyphens before the lookup);
* options declared with an argument consume the next token (which may start with ``-``
  when it is a number, e.g. ``-min -1``);
* boolean flags take no value;
* an unknown option is an error (``UDFArgumentException``);
* ``-help`` raises ``UDFArgumentException`` carrying the usage text.
"""
from __future__ import annotations

import shlex
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable


class UDFArgumentException(ValueError):
    """Raised for malformed arguments / option strings (Hive's UDFArgumentException)."""


@dataclass
class Opt:
    name: str                      # short name, e.g. "iters"
    long: str | None = None        # long name, e.g. "iterations"
    has_arg: bool = True
    default: Any = None
    type: Callable[[str], Any] = str
    help: str = ""
    aliases: tuple = ()
    inert: str = ""                # non-empty: accepted for compatibility, has no effect (why)

    def names(self) -> list[str]:
        out = [self.name]
        if self.long:
            out.append(self.long)
        out.extend(self.aliases)
        return out


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "on")


def flag(name: str, long: str | None = None, help: str = "", aliases: tuple = (),
         inert: str = "") -> Opt:
    return Opt(name, long, has_arg=False, default=False, type=_bool, help=help, aliases=aliases,
               inert=inert)


def opt(name: str, long: str | None = None, default: Any = None, type: Callable = str,
        help: str = "", aliases: tuple = (), inert: str = "") -> Opt:
    return Opt(name, long, has_arg=True, default=default, type=type, help=help, aliases=aliases,
               inert=inert)


_warned: set = set()


def warn_inert(func_name: str, o: Opt) -> None:
    """Log (once per function and option) that an accepted option has no effect here."""
    key = (func_name, o.name)
    if key in _warned:
        return
    _warned.add(key)
    import logging

    logging.getLogger("hivemall_amd").warning("%s: option -%s is accepted for compatibility but "
                                              "has no effect: %s", func_name, o.name, o.inert)


class Options:
    """A set of declared options (the ``getOptions()`` of a Hivemall UDF)."""

    def __init__(self, opts: Iterable[Opt] = (), func_name: str = "function"):
        self.func_name = func_name
        self._opts: list[Opt] = []
        self._lookup: dict[str, Opt] = {}
        for o in opts:
            self.add(o)
        if "help" not in self._lookup:
            self.add(flag("help", help="Show function help"))

    def add(self, o: Opt) -> "Options":
        for n in o.names():
            if n in self._lookup and self._lookup[n] is not o:
                raise ValueError(f"duplicate option name: {n}")
            self._lookup[n] = o
        self._opts.append(o)
        return self

    def extend(self, opts: Iterable[Opt]) -> "Options":
        for o in opts:
            if o.name in self._lookup:
                continue
            self.add(o)
        return self

    def copy(self, func_name: str | None = None) -> "Options":
        return Options(list(self._opts), func_name or self.func_name)

    def usage(self) -> str:
        lines = [f"usage: {self.func_name}"]
        for o in self._opts:
            spell = f"-{o.name}"
            if o.long:
                spell += f",--{o.long}"
            if o.has_arg:
                spell += f" <arg>"
            d = f" (default: {o.default})" if o.has_arg and o.default is not None else ""
            inert = f" [no effect: {o.inert}]" if o.inert else ""
            lines.append(f" {spell:<32} {o.help}{d}{inert}")
        return "\n".join(lines)

    def parse(self, optstr: str | None) -> "CommandLine":
        values: dict[str, Any] = {}
        present: set[str] = set()
        tokens = _tokenize(optstr)
        i = 0
        while i < len(tokens):
            tok = tokens[i]
            if not tok.startswith("-") or tok in ("-", "--"):
                raise UDFArgumentException(
                    f"{self.func_name}: unexpected argument '{tok}' in option string '{optstr}'")
            key = tok.lstrip("-")
            val_inline = None
            if "=" in key and key.split("=", 1)[0] in self._lookup:
                key, val_inline = key.split("=", 1)
            o = self._lookup.get(key)
            if o is None:
                raise UDFArgumentException(
                    f"{self.func_name}: Unrecognized option: {tok}\n{self.usage()}")
            if o.name == "help":
                raise UDFArgumentException(self.usage())
            present.add(o.name)
            if o.inert:
                warn_inert(self.func_name, o)
            if o.has_arg:
                if val_inline is not None:
                    raw = val_inline
                else:
                    if i + 1 >= len(tokens):
                        raise UDFArgumentException(
                            f"{self.func_name}: Missing argument for option: {o.name}")
                    raw = tokens[i + 1]
                    i += 1
                try:
                    values[o.name] = o.type(raw)
                except (TypeError, ValueError) as e:
                    raise UDFArgumentException(
                        f"{self.func_name}: invalid value '{raw}' for -{o.name}: {e}") from e
            else:
                values[o.name] = True
            i += 1
        return CommandLine(self, values, present)


def _tokenize(optstr: str | None) -> list[str]:
    if optstr is None:
        return []
    s = str(optstr).strip()
    if not s:
        return []
    try:
        return shlex.split(s)
    except ValueError:
        return s.split()


@dataclass
class CommandLine:
    spec: Options
    values: dict = field(default_factory=dict)
    present: set = field(default_factory=set)

    def has(self, name: str) -> bool:
        o = self.spec._lookup.get(name)
        return o is not None and o.name in self.present

    def get(self, name: str, default: Any = None) -> Any:
        o = self.spec._lookup.get(name)
        if o is None:
            raise KeyError(name)
        if o.name in self.values:
            return self.values[o.name]
        if default is not None:
            return default
        return o.default

    def __getitem__(self, name: str) -> Any:
        return self.get(name)

    def as_dict(self) -> dict:
        return {o.name: self.get(o.name) for o in self.spec._opts if o.name != "help"}
