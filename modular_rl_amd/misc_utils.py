"""Config / CLI plumbing and small utilities with the reference's names and meaning
(`misc_utils.py:51-104,134-189`).  Host-side Python by nature (argparse), not
compute."""
from collections import defaultdict  # noqa: F401  (re-exported like the reference)

import numpy as np


class dict2(dict):
    """dictionary-like object that exposes its keys as attributes (`misc_utils.py:139-143`)."""

    def __init__(self, **kwargs):
        dict.__init__(self, kwargs)
        self.__dict__ = self


def update_default_config(tuples, usercfg):
    """Defaults from (name, type, default, desc) tuples, overridden by usercfg (`misc_utils.py:56-74`)."""
    out = dict2()
    for (name, _, defval, _) in tuples:
        out[name] = defval
    if usercfg:
        for (k, v) in usercfg.items():
            if k in out:
                out[k] = v
    return out


def update_argument_parser(parser, options, **kwargs):
    """Add --name flags for option tuples (`misc_utils.py:76-85`)."""
    kwargs = kwargs.copy()
    for (name, typ, default, desc) in options:
        flag = "--" + name
        if flag in parser._option_string_actions.keys():  # pylint: disable=W0212
            print("warning: already have option %s. skipping" % name)
        else:
            parser.add_argument(flag, type=typ, default=kwargs.pop(name, default), help=desc or " ")
    if kwargs:
        raise ValueError("options %s ignored" % kwargs)


def comma_sep_ints(s):
    """'64,64' -> [64, 64].  The reference returns a one-shot ``map`` under py3
    (`misc_utils.py:87-91`); a list is the intended behaviour."""
    if s:
        return [int(v) for v in s.split(",")]
    return []


def IDENTITY(x):
    return x


GENERAL_OPTIONS = [
    ("seed", int, 0, "random seed"),
    ("metadata", str, "", "metadata about experiment"),
    ("outfile", str, "./tmp/a.h5", "output file"),
    ("use_hdf", int, 0, "whether to make an hdf5 file with results and snapshots"),
    ("snapshot_every", int, 0, "how often to snapshot"),
    ("load_snapshot", str, "", "path to snapshot"),
    ("video", int, 1, "whether to record video"),
]


def zipsame(*seqs):
    L = len(seqs[0])
    assert all(len(seq) == L for seq in seqs[1:])
    return zip(*seqs)


def flatten(arrs):
    return np.concatenate([np.asarray(arr).ravel() for arr in arrs])


def unflatten(vec, shapes):
    i = 0
    arrs = []
    for shape in shapes:
        size = int(np.prod(shape))
        arrs.append(vec[i:i + size].reshape(shape))
        i += size
    return arrs


class EzPickle:
    """Objects pickled via their constructor arguments (`misc_utils.py:163-189`)."""

    def __init__(self, *args, **kwargs):
        self._ezpickle_args = args
        self._ezpickle_kwargs = kwargs

    def __getstate__(self):
        return {"_ezpickle_args": self._ezpickle_args, "_ezpickle_kwargs": self._ezpickle_kwargs}

    def __setstate__(self, d):
        out = type(self)(*d["_ezpickle_args"], **d["_ezpickle_kwargs"])
        self.__dict__.update(out.__dict__)


def fmt_row(width, row, header=False):
    out = " | ".join(fmt_item(x, width) for x in row)
    if header:
        out = out + "\n" + "-" * len(out)
    return out


def fmt_item(x, l):
    if isinstance(x, np.ndarray):
        assert x.ndim == 0
        x = x.item()
    rep = "%g" % x if isinstance(x, float) else str(x)
    return " " * (l - len(rep)) + rep
