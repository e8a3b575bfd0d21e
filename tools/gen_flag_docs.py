#!/usr/bin/env python3
"""Generate docs/parameters.md from the live argument parser (so the table never drifts).

usage: python tools/gen_flag_docs.py > docs/parameters.md
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hetseq_amd import options  # noqa: E402


def rows(parser):
    for g in parser._action_groups:
        acts = [a for a in g._group_actions if not isinstance(a, argparse._HelpAction)]
        if not acts:
            continue
        yield g.title, acts


def fmt_default(a):
    if isinstance(a, (argparse._StoreTrueAction, argparse._StoreFalseAction)):
        return "flag"
    d = a.default
    return "`%r`" % (d,) if d is not None else "None"


def main():
    out = ["# Command-line parameters", "",
           "Generated from `hetseq_amd/options.py` by `tools/gen_flag_docs.py`.  The flag set, names,",
           "aliases and defaults follow the reference parser (`options.py:5-290`); the last group holds",
           "the MI355X extensions, which never change a reference default.", ""]
    for task, opt in (("bert", "adam"), ("mnist", "adadelta")):
        p = options.get_training_parser(task=task, optimizer=opt)
        out.append("## `--task %s --optimizer %s`" % (task, opt))
        out.append("")
        for title, acts in rows(p):
            out.append("### %s" % title)
            out.append("")
            out.append("| flag | default | choices | help |")
            out.append("|---|---|---|---|")
            for a in acts:
                names = ", ".join("`%s`" % s for s in a.option_strings)
                ch = ", ".join(str(c) for c in a.choices) if a.choices else ""
                hp = (a.help or "").replace("|", "/").replace("\n", " ")
                out.append("| %s | %s | %s | %s |" % (names, fmt_default(a), ch, hp))
            out.append("")
    print("\n".join(out))


if __name__ == "__main__":
    main()
