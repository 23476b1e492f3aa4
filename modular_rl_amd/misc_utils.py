"""Option-tuple config and CLI plumbing behind the reference's agent API.

The reference configures everything through ``(name, type, default, help)`` tuples
(``misc_utils.py:56-104``): agents merge user settings over the defaults and
``run_pg.py`` turns the same tuples into ``--name`` flags.  Only the pieces the
product imports live here: ``update_default_config``, ``update_argument_parser``,
``comma_sep_ints``, ``IDENTITY`` and ``GENERAL_OPTIONS``.
"""


class Config(dict):
    """A dict whose keys read as attributes too (``cfg["gamma"]`` == ``cfg.gamma``),
    the behaviour of the reference's ``dict2`` (``misc_utils.py:139-143``)."""

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as exc:
            raise AttributeError(key) from exc

    def __setattr__(self, key, value):
        self[key] = value


def update_default_config(option_tuples, usercfg):
    """Defaults of ``option_tuples`` overridden by the user's values for KNOWN names;
    unknown user keys are dropped (``misc_utils.py:56-74``)."""
    cfg = Config((opt[0], opt[2]) for opt in option_tuples)
    for key, value in (usercfg or {}).items():
        if key in cfg:
            cfg[key] = value
    return cfg


def update_argument_parser(parser, option_tuples, **overrides):
    """Register ``--name`` for every option tuple; a flag already registered by an
    earlier group is skipped with a warning, and an override naming no tuple is an
    error (``misc_utils.py:76-85``)."""
    pending = dict(overrides)
    for name, typ, default, helptext in option_tuples:
        flag = f"--{name}"
        if flag in parser._option_string_actions:  # pylint: disable=protected-access
            print(f"warning: already have option {name}. skipping")
            continue
        parser.add_argument(flag, type=typ, default=pending.pop(name, default), help=helptext or " ")
    if pending:
        raise ValueError(f"options {pending} ignored")


def comma_sep_ints(text):
    """``"64,64"`` -> ``[64, 64]``.  The reference returns a one-shot ``map`` under
    py3 (``misc_utils.py:87-91``), which would leave the VF net
    with no hidden layers; a list is the intended behaviour."""
    return [int(tok) for tok in text.split(",")] if text else []


def IDENTITY(x):  # noqa: N802  (the reference's name: agentzoo filters default to it)
    return x


# run_pg.py's general flags (misc_utils.py:96-104)
GENERAL_OPTIONS = [
    ("seed", int, 0, "random seed"),
    ("metadata", str, "", "metadata about experiment"),
    ("outfile", str, "./tmp/a.h5", "output file"),
    ("use_hdf", int, 0, "whether to make an hdf5 file with results and snapshots"),
    ("snapshot_every", int, 0, "how often to snapshot"),
    ("load_snapshot", str, "", "path to snapshot"),
    ("video", int, 1, "whether to record video"),
]
