"""Attribute helpers used by the name lookup of create_model / activation_wrapper (reference utils/attr.py)."""
import functools


def rgetattr(obj, attr, *args):
    return functools.reduce(lambda o, a: getattr(o, a, *args), [obj] + attr.split("."))


def rsetattr(obj, attr, val):
    pre, _, post = attr.rpartition(".")
    return setattr(rgetattr(obj, pre) if pre else obj, post, val)


def getattr_nested(obj, path):
    try:
        return functools.reduce(getattr, path.split("."), obj)
    except AttributeError:
        return False
