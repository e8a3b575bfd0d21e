"""Fault injection for failure-handling tests.

``HETSEQ_FAULT`` holds ``;``-separated actions, each ``kind:RANK@UPDATE[:ARG]``:

* ``kill:1@3``        rank 1 exits (``os._exit(17)``) at the start of update 3
* ``raise:0@2``       rank 0 raises ``InjectedFault`` at the start of update 2
* ``delay:1@5:2.5``   rank 1 sleeps 2.5 s at the start of update 5 (straggler)

A killed or stalled rank must turn into a bounded-time error on the others
(``--collective-timeout``), never a silent hang; ``tests/test_faults_cpu.py``
checks that with gloo.  Without the variable this module costs one dict lookup
per update.
"""
import os
import time


class InjectedFault(RuntimeError):
    pass


def _parse(spec):
    acts = []
    for item in filter(None, (x.strip() for x in spec.split(";"))):
        kind, rest = item.split(":", 1)
        where, _, arg = rest.partition(":")
        rank, upd = where.split("@")
        acts.append((kind, int(rank), int(upd), arg))
    return acts


_ACTS = None


def maybe_inject(rank, num_updates):
    global _ACTS
    if _ACTS is None:
        _ACTS = _parse(os.environ.get("HETSEQ_FAULT", ""))
    for kind, r, u, arg in _ACTS:
        if r != rank or u != num_updates:
            continue
        if kind == "kill":
            print("| fault injection: rank %d exiting at update %d" % (rank, num_updates), flush=True)
            os._exit(17)
        elif kind == "raise":
            raise InjectedFault("injected fault on rank %d at update %d" % (rank, num_updates))
        elif kind == "delay":
            time.sleep(float(arg or 1.0))
        else:
            raise ValueError("unknown HETSEQ_FAULT action %r" % kind)
