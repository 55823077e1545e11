"""CSV column names -- mirrors ``rss_simulator/column_names.py:4-12``.

The four input columns of a 4-tuple CSV, then the two columns ``Simulator.calc_hash`` /
``calc_queue_number`` append.  Built with Enum's functional API: member ``X`` has value
``x`` (lower-case), exactly as the reference's class body spells them out.
"""
from enum import Enum

_INPUT = ("src_ip", "dst_ip", "src_port", "dst_port")
_OUTPUT = ("hash_result", "queue_number")

ColumnNames = Enum("ColumnNames", [(name.upper(), name) for name in _INPUT + _OUTPUT],
                   module=__name__, qualname="ColumnNames")
ColumnNames.__doc__ = "Column names of the 4-tuple CSV and of the two columns the simulator adds."

INPUT_COLUMNS = tuple(ColumnNames(name) for name in _INPUT)
