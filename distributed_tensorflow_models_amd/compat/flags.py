"""``tf.app.flags`` / ``tf.app.run`` facade.

Flags are module-level globals defined as a side effect of importing modules (exactly like the
reference, where a script's flag set is the union of its imports), parsed from argv by ``run``.
Accepts ``--name=value``, ``--name value``, ``--bool`` / ``--nobool``.
"""
import sys


class _FlagValues:
    def __init__(self):
        object.__setattr__(self, "_defs", {})
        object.__setattr__(self, "_vals", {})
        object.__setattr__(self, "_parsed", False)

    def _define(self, name, default, help_, kind):
        self._defs[name] = (default, help_, kind)
        self._vals.setdefault(name, default)

    def __getattr__(self, name):
        vals = object.__getattribute__(self, "_vals")
        if name in vals:
            return vals[name]
        raise AttributeError("unknown flag --%s" % name)

    def __setattr__(self, name, value):
        if name not in self._defs:
            raise AttributeError("unknown flag --%s" % name)
        self._vals[name] = value

    def __contains__(self, name):
        return name in self._defs

    def _convert(self, name, raw):
        default, _h, kind = self._defs[name]
        if kind == "bool":
            return str(raw).lower() in ("1", "true", "t", "yes", "y")
        if kind == "int":
            return int(float(raw)) if isinstance(raw, str) and ("e" in raw.lower() or "." in raw) else int(raw)
        if kind == "float":
            return float(raw)
        if kind == "list":
            return [s for s in str(raw).split(",") if s]
        return raw

    def parse(self, argv, known_only=True):
        rest = [argv[0]] if argv else []
        i = 1
        while i < len(argv):
            a = argv[i]
            if a.startswith("--") and len(a) > 2:
                body = a[2:]
                if "=" in body:
                    name, val = body.split("=", 1)
                    name = name.replace("-", "_")
                    if name in self._defs:
                        self._vals[name] = self._convert(name, val)
                        i += 1
                        continue
                else:
                    name = body.replace("-", "_")
                    if name in self._defs:
                        if self._defs[name][2] == "bool":
                            self._vals[name] = True
                            i += 1
                            continue
                        if i + 1 < len(argv):
                            self._vals[name] = self._convert(name, argv[i + 1])
                            i += 2
                            continue
                    if name.startswith("no") and name[2:] in self._defs and self._defs[name[2:]][2] == "bool":
                        self._vals[name[2:]] = False
                        i += 1
                        continue
                if not known_only:
                    raise ValueError("unknown flag %s" % a)
            rest.append(a)
            i += 1
        object.__setattr__(self, "_parsed", True)
        return rest

    def flag_values_dict(self):
        return dict(self._vals)

    def help_text(self):
        lines = []
        for n, (d, h, k) in sorted(self._defs.items()):
            lines.append("  --%s (%s, default %r): %s" % (n, k, d, h))
        return "\n".join(lines)

    def reset(self, name=None):
        if name is None:
            for n, (d, _h, _k) in self._defs.items():
                self._vals[n] = d
        else:
            self._vals[name] = self._defs[name][0]


FLAGS = _FlagValues()


def DEFINE_string(name, default, help=""):  # noqa: N802,A002
    FLAGS._define(name, default, help, "string")


def DEFINE_integer(name, default, help=""):  # noqa: N802,A002
    FLAGS._define(name, default, help, "int")


def DEFINE_float(name, default, help=""):  # noqa: N802,A002
    FLAGS._define(name, default, help, "float")


def DEFINE_boolean(name, default, help=""):  # noqa: N802,A002
    FLAGS._define(name, default, help, "bool")


DEFINE_bool = DEFINE_boolean


def DEFINE_list(name, default, help=""):  # noqa: N802,A002
    FLAGS._define(name, default, help, "list")


def run(main=None, argv=None):
    """tf.app.run: parse flags from argv, then call main(argv)."""
    argv = list(sys.argv if argv is None else argv)
    if "--help" in argv or "-h" in argv:
        print("flags:\n" + FLAGS.help_text())
        sys.exit(0)
    rest = FLAGS.parse(argv)
    if main is None:
        main = sys.modules["__main__"].main
    sys.exit(main(rest))
