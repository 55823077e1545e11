"""Histogram output mode -- counterpart of ``Simulator.show_histogram``
(``rss_simulator/simulator.py:118-172``), drawn from the device per-queue histogram.

Same figure content as the reference (pinned by ``tests/golden/histogram.json``): one
bar per queue over ``[0, Q)`` (bin i at ``i + 0.05``, width 0.9 -- what
``df.hist(bins=Q, range=[0, Q], rwidth=0.9)`` draws), the title / axis labels, and
the four-line caption with the key (split at character 94), the hash-table size,
the number of queues and the number of non-empty queues.  ``output`` saves a PNG
(headless use); otherwise ``plt.show()`` as in the reference.
"""
import numpy as np

TITLE = "Number of Unique Flows per Queue"
XLABEL = "Queue Number"
YLABEL = "Number of Flows"


def caption(hash_key_str, hash_table_size, num_queues, counts):
    """The caption text of ``simulator.py:160-169``."""
    key_str = "Hash Key: {}\n{}{}".format(hash_key_str[:94], " " * 17, hash_key_str[94:])
    return "\n".join([
        key_str,
        "Hash Table Size: {}".format(hash_table_size),
        "Number Queues: {}".format(num_queues),
        "Number of Queues Chosen by Hash Function: {}".format(int(np.count_nonzero(counts))),
    ])


def figure(counts, hash_key_str, hash_table_size, num_queues):
    """Build (and return) the matplotlib figure for per-queue ``counts``."""
    import matplotlib.pyplot as plt
    from matplotlib.ticker import MaxNLocator

    counts = np.asarray(counts, dtype=np.float64)
    if len(counts) < num_queues:  # queues >= min(htable, 2**32) are never chosen
        counts = np.concatenate([counts, np.zeros(num_queues - len(counts))])
    fig, ax = plt.subplots(figsize=(12, 8))
    ax.bar(np.arange(num_queues) + 0.05, counts, width=0.9, align="edge", color="#86bf91",
           zorder=2)
    for side in ("right", "top", "left"):
        ax.spines[side].set_visible(False)
    ax.tick_params(axis="both", which="both", bottom=False, top=False, left=False, right=False)
    for tick in ax.get_yticks():
        ax.axhline(y=tick, linestyle="dashed", alpha=0.8, color="#dddddd", zorder=1)
    ax.set_title(TITLE, weight="bold", size=16)
    ax.set_xlabel(XLABEL, labelpad=20, weight="bold", size=12)
    ax.set_ylabel(YLABEL, labelpad=20, weight="bold", size=12)
    ax.yaxis.set_major_locator(MaxNLocator(integer=True))
    ax.set_xlim(0, num_queues)
    fig.text(0.04, 0.03, caption(hash_key_str, hash_table_size, num_queues, counts), fontsize=12)
    fig.subplots_adjust(bottom=0.27)
    return fig


def show(counts, hash_key_str, hash_table_size, num_queues, output=None):
    """Display the histogram (``plt.show()``) or, with ``output``, save it as a PNG."""
    import matplotlib.pyplot as plt

    fig = figure(counts, hash_key_str, hash_table_size, num_queues)
    if output:
        fig.savefig(output)
        plt.close(fig)
    else:
        plt.show()
