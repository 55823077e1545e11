"""Positive-int argparse type (``rss_simulator/arg_parse_types/positive_int.py:8-30``).

Used for ``--hash-table-size`` / ``--num-queues``; an argument that ``int()`` rejects
reports ``int()``'s own message, one below 1 reports ``"Number must be positive."``.
"""
from argparse import ArgumentTypeError

_NOT_POSITIVE = "Number must be positive."


def _to_int(text):
    try:
        return int(text)
    except ValueError as err:
        raise ArgumentTypeError(err)


class PositiveInt(object):
    """Namespace for the ``parse`` callable handed to argparse."""

    @staticmethod
    def parse(arg):
        value = _to_int(arg)
        if value >= 1:
            return value
        raise ArgumentTypeError(_NOT_POSITIVE)
