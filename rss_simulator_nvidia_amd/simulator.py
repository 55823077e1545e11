"""RSS simulator driver -- drop-in for ``rss_simulator/simulator.py`` (``Simulator``).

Public methods and their behaviour follow the reference:

* ``load_ips_from_csv``  (``simulator.py:43-72``): ``pd.read_csv``, the same
  ``ParseException`` messages (the unreadable-file message keeps the reference's
  literal, unformatted ``'{csv}'``);
* ``calc_hash``          (``simulator.py:74-92``): adds the int64 ``hash_result``
  column.  Here the whole column is one kernel launch that also produces the
  queue column and the per-queue histogram;
* ``calc_queue_number``  (``simulator.py:94-98``): adds ``queue_number`` =
  ``hash_result % htable % queues`` (computed by the same kernel pass);
* ``write_statistics``   (``simulator.py:100-116``): ``queue_number,counts`` rows
  for the non-empty queues (from the device histogram), then the full table,
  then the same stdout line;
* ``show_histogram``     (``simulator.py:118-172``): the per-queue bar chart with
  the key / htable / queue caption (``histogram.py``; ``output=`` saves a PNG).
"""
from __future__ import print_function

import numpy as np
import pandas as pd
from pandas.errors import ParserError as pd_ParserError

from rss_simulator_nvidia_amd import _native, histogram
from rss_simulator_nvidia_amd.column_names import INPUT_COLUMNS, ColumnNames
from rss_simulator_nvidia_amd.exceptions import ParseException
from rss_simulator_nvidia_amd.ingest import pack_frame, pack_frame6
from rss_simulator_nvidia_amd.toeplitz import Toeplitz

_HASH = ColumnNames.HASH_RESULT.value
_QUEUE = ColumnNames.QUEUE_NUMBER.value


def _read_canonical_csv(path):
    """The DataFrame ``pd.read_csv(path)`` would build, for a canonical 4-tuple file (header =
    the four input columns in any order, dotted quads, decimal ports: ``rss_csv_parse``),
    read by pyarrow; None for anything else (unreadable, not canonical, no pyarrow), which
    the caller hands to pandas."""
    try:
        import pyarrow as pa
        import pyarrow.csv as pacsv
        with open(path, "rb") as f:
            data = f.read()
    except (ImportError, OSError, TypeError, ValueError):
        return None
    if _native.csv_parse(data) is None:  # not canonical
        return None
    try:
        df = pacsv.read_csv(pa.BufferReader(data)).to_pandas()
    except Exception:  # (pandas then reads it -- and raises -- as the reference)
        return None
    names = {c.value for c in INPUT_COLUMNS}
    if set(df.columns) != names or len(df.columns) != 4 or any(
            df[c.value].dtype != (object if c.value.endswith("_ip") else np.int64)
            for c in INPUT_COLUMNS):
        return None
    return df


class Simulator(object):
    """RSS simulator class (``simulator.py:26``)."""

    def __init__(self, hash_key, hash_table_size, queue_number, hash_fields=None, ipv6=False,
                 reta=None, devices=None):
        """Key as ``List[int]``, hash-table size and number of queues (both >= 1).

        Additive options: ``hash_fields`` (mask or ``'sdfn'``
        letters) selects the hashed fields; ``ipv6`` reads IPv6 address columns; ``reta``
        (``hash_table_size`` queue ids) replaces ``bucket % queue_number``; ``devices``
        (GPU ids) splits ``calc_hash``'s rows over several GPUs, one context each (the
        default hashes on one GPU).  Results do not depend on ``devices``."""
        self.__ip_df = None
        self.__toeplitz = Toeplitz(hash_key, hash_fields or "sdfn")
        self.__ipv6 = ipv6
        self.__reta = reta
        self.__devices = None if devices is None else tuple(int(d) for d in devices)
        if self.__devices == ():
            raise ValueError("devices must name at least one GPU")
        self.__hash_table_size = hash_table_size
        self.__queue_num = queue_number
        self.__queues = None
        self.__counts = None
        self.__count_rows = None  # sparse (queue, count) rows when queues are the hashes

    @property
    def data_frame(self):
        """The working DataFrame (input columns + the columns added so far)."""
        return self.__ip_df

    @property
    def queue_counts(self):
        """uint64[num_queues] per-queue counts from the last ``calc_hash``."""
        return self.__counts

    def load_ips_from_csv(self, csv_path):
        """Read the 4-tuple CSV; raise ParseException like ``simulator.py:54-71``.

        A canonical file (the CSV fast path's format, checked by ``rss_csv_parse``) is read by
        pyarrow's multi-threaded reader into the same DataFrame ``pd.read_csv`` builds (str
        address columns, int64 ports, header order) in ~half the time; any other file, and
        every error, takes ``pd.read_csv`` as the reference does."""
        df = _read_canonical_csv(csv_path)
        if df is not None:
            self.load_frame(df)
            return
        try:
            df = pd.read_csv(csv_path)
        except (UnicodeDecodeError, IOError, pd_ParserError):
            msg = "Couldn't parse '{csv}' file, make sure it's a valid CSV encoded with 'utf-8'"
            raise ParseException(msg)
        expected = {col.value for col in INPUT_COLUMNS}
        missing_columns = expected - set(df.columns.tolist())
        if missing_columns:
            raise ParseException("{csv} is missing columns: {cols}".format(
                csv=csv_path, cols=", ".join(missing_columns)))
        self.load_frame(df)

    def load_frame(self, df):
        """Use an in-memory DataFrame (same column contract as the CSV)."""
        self.__ip_df = df
        self.__queues = None
        self.__counts = None
        self.__count_rows = None

    def calc_hash(self):
        """Hash every row on the GPU and add the ``hash_result`` column."""
        df = self.__ip_df
        if len(df) == 0:
            # the reference's DataFrame.apply on zero rows fails the same way
            raise ValueError("Cannot set a DataFrame with multiple columns to the single column "
                             "hash_result")
        H, Q = self.__hash_table_size, self.__queue_num
        sparse = _native.queues_are_hashes(H, Q, self.__reta)
        if sparse:  # H, Q >= 2**32: hash % H % Q = hash (simulator.py:97); hashes only
            H = Q = 1
        if self.__ipv6:
            h, q, c = self.__toeplitz.compute_queues6(pack_frame6(df), H, Q, self.__reta,
                                                      self.__devices)
        else:
            h, q, c = self.__toeplitz.compute_queues(pack_frame(df), H, Q, self.__reta,
                                                     self.__devices)
        df[_HASH] = h.astype(np.int64)
        self.__count_rows = None
        if sparse:  # a 2**32-entry histogram: the non-empty queues only (value_counts)
            q, c = h, None
            values, freq = np.unique(h, return_counts=True)
            self.__count_rows = [(int(v), int(f)) for v, f in zip(values, freq)]
        self.__queues = q
        self.__counts = c

    def calc_queue_number(self):
        """Add ``queue_number`` = ``hash_result % htable % queues`` (``simulator.py:96-98``)."""
        if self.__queues is None:
            raise AttributeError("'DataFrame' object has no attribute 'hash_result'")
        self.__ip_df[_QUEUE] = self.__queues.astype(np.int64)

    def queue_count_rows(self):
        """``[(queue, count)]`` for non-empty queues, ascending (value_counts().sort_index())."""
        if self.__count_rows is not None:
            return self.__count_rows
        counts = self.__counts
        nz = np.flatnonzero(counts)
        return [(int(q), int(counts[q])) for q in nz]

    def write_statistics(self, output):
        """Write counts then the full table to ``output`` (``simulator.py:100-116``).

        A frame of exactly the four input columns (any order) + ``hash_result`` +
        ``queue_number`` whose cells are canonical (quads with octets 0..255 and no leading
        zeros, integer ports 0..65535 -- text pandas writes back unchanged) is written by the
        native formatter (``rss_csv_format``, the bytes ``to_csv`` would write, ~8x faster);
        any other frame by pandas, as the reference."""
        if not self.__write_native(output):
            with open(output, "w") as f:
                f.write("{},counts\n".format(_QUEUE))
                for q, c in self.queue_count_rows():
                    f.write("{},{}\n".format(q, c))
            self.__ip_df.to_csv(output, mode="a", index=False)
        print("Wrote statistics to {csv}.".format(csv=output))

    def __write_native(self, output):
        """The canonical-frame path of :meth:`write_statistics`; False when it does not apply."""
        df, counts = self.__ip_df, self.__counts
        names = [c.value for c in INPUT_COLUMNS]
        cols = list(df.columns)
        if (counts is None or self.__count_rows is not None or len(df) == 0 or len(cols) != 6
                or sorted(cols[:4]) != sorted(names) or cols[4:] != [_HASH, _QUEUE]):
            return False
        packed = {}
        for name in names[:2]:
            values = df[name].to_numpy()
            if pd.api.types.infer_dtype(values, skipna=False) != "string":
                return False
            parsed = _native.parse_dotted(values.tolist(), canonical=True)
            if parsed is None or not parsed[0].all():
                return False
            packed[name] = parsed[1]
        for name in names[2:] + [_HASH, _QUEUE]:
            col = df[name]
            top = 0xFFFF if name in names[2:] else 0xFFFFFFFF
            if col.dtype.kind not in "iu" or col.min() < 0 or col.max() > top:
                return False
            packed[name] = col.to_numpy().astype(np.uint32)
        tuples = np.empty(len(df), dtype=_native.TUPLE_DTYPE)
        tuples["sip"], tuples["dip"] = packed[names[0]], packed[names[1]]
        tuples["ports"] = (packed[names[2]] << np.uint32(16)) | packed[names[3]]
        layout = _native.RssCsvLayout()
        for f, name in enumerate(cols[:4]):
            layout.field_column[f] = names.index(name)
        image = _native.csv_format(tuples, packed[_HASH], packed[_QUEUE],
                                   np.asarray(counts, dtype=np.uint64), layout)
        with open(output, "wb") as f:
            f.write(memoryview(image))
        return True

    def histogram_caption(self):
        """The caption lines of ``simulator.py:160-169``."""
        return histogram.caption(self.__toeplitz.hash_key_str(), self.__hash_table_size,
                                 self.__queue_num, self.__counts)

    def show_histogram(self, output=None):
        """Per-queue bar chart + caption (``simulator.py:118-172``); PNG if ``output``."""
        histogram.show(self.__counts, self.__toeplitz.hash_key_str(), self.__hash_table_size,
                       self.__queue_num, output)
