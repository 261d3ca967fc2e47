"""tf.logging facade (reference e.g. alexnet/cifar10_alexnet_bsp.py:16 set_verbosity(INFO))."""
import logging as _logging
import sys

DEBUG, INFO, WARN, ERROR, FATAL = _logging.DEBUG, _logging.INFO, _logging.WARNING, _logging.ERROR, _logging.CRITICAL
_log = _logging.getLogger("dtm")
if not _log.handlers:
    _h = _logging.StreamHandler(sys.stderr)
    _h.setFormatter(_logging.Formatter("%(levelname).1s%(asctime)s %(message)s", "%m%d %H:%M:%S"))
    _log.addHandler(_h)
    _log.setLevel(INFO)
    _log.propagate = False


def set_verbosity(v):
    _log.setLevel(v)


def info(msg, *a):
    _log.info(msg, *a)


def warning(msg, *a):
    _log.warning(msg, *a)


warn = warning


def error(msg, *a):
    _log.error(msg, *a)


def debug(msg, *a):
    _log.debug(msg, *a)


def fatal(msg, *a):
    _log.critical(msg, *a)
    raise SystemExit(1)
