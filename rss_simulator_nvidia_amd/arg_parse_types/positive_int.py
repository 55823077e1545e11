"""Positive-int argparse type (``rss_simulator/arg_parse_types/positive_int.py:8-30``)."""
from argparse import ArgumentTypeError


class PositiveInt(object):
    """Positive int argument class."""

    @staticmethod
    def parse(arg):
        """Parse ``arg`` with ``int()`` and require a value >= 1.

        Messages match the reference: ``int()``'s own ValueError text, or
        ``"Number must be positive."``.
        """
        try:
            num = int(arg)
        except ValueError as v_err:
            raise ArgumentTypeError(v_err)
        if num < 1:
            raise ArgumentTypeError("Number must be positive.")
        return num
