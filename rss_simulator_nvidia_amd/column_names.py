"""CSV column names -- mirrors ``rss_simulator/column_names.py:4-12``."""
from enum import Enum


class ColumnNames(Enum):
    """Column names of the 4-tuple CSV and of the two columns the simulator adds."""

    SRC_IP = "src_ip"
    DST_IP = "dst_ip"
    SRC_PORT = "src_port"
    DST_PORT = "dst_port"
    HASH_RESULT = "hash_result"
    QUEUE_NUMBER = "queue_number"


INPUT_COLUMNS = (ColumnNames.SRC_IP, ColumnNames.DST_IP, ColumnNames.SRC_PORT, ColumnNames.DST_PORT)
