"""Callables for argparse's ``type=``: ``PositiveInt.parse`` for the table/queue sizes and
the decorator that turns a parser's exception into ``ArgumentTypeError`` (the reference's
``arg_parse_types`` package)."""
from . import arg_parse_type_decorator as _decorator_module
from . import positive_int as _positive_int_module

arg_parse_type_decorator = _decorator_module.arg_parse_type_decorator
PositiveInt = _positive_int_module.PositiveInt

__all__ = ["PositiveInt", "arg_parse_type_decorator"]
