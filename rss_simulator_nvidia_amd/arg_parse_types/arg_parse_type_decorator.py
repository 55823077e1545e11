"""Wrap a parse function for argparse (``arg_parse_type_decorator.py:5-20``).

Any exception the wrapped function raises becomes ``ArgumentTypeError`` so that
argparse reports ``error: argument --x: <message>`` and exits with status 2.
"""
from argparse import ArgumentTypeError
from functools import wraps


def arg_parse_type_decorator(parse_func):
    """Return ``parse_func`` with every exception re-raised as ArgumentTypeError."""
    @wraps(parse_func)
    def _parse(arg):
        try:
            return parse_func(arg)
        except Exception as ex:  # noqa: BLE001 -- same catch-all as the reference
            raise ArgumentTypeError(ex)
    return _parse
