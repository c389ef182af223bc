"""Rundir / params.json helpers with the reference's semantics (tools/setup/meta.py:11-52), so the
drop-in plugin's CLI can register itself in a rundir without importing the reference.

  rundir(args)          --rundir, else the last line of stdin (the previous pipeline stage's output)
  params(rundir, name)  params.json (or one section of it)
  load(rundir, file)    any JSON file of the rundir
  extend(rundir, name, section)   add ONE new section; refuses to overwrite (meta.py:47)
"""
import json
import os
import sys


def rundir(args):
    assert hasattr(args, "rundir"), "Invalid args inputs, should have 'rundir' attribute set by ArgumentParser"
    if args.rundir is None:
        lines = sys.stdin.readlines()
        assert len(lines) >= 1, "Invalid standard output from previous process: expected RUNDIR on last line."
        path = lines[-1].split("\n")[0]
    else:
        path = args.rundir
    assert os.path.exists(path), "Invalid run directory '{}'".format(path)
    return path


def params(rundir, name=None):
    path = os.path.join(rundir, "params.json")
    p = {}
    if os.path.exists(path):
        with open(path) as f:
            p = json.load(f)
    if name is None:
        return p
    assert name in p, "Invalid property name {} for params.json object".format(name)
    return p[name]


def load(rundir, filename):
    with open(os.path.join(rundir, filename)) as f:
        return json.load(f)


def extend(rundir, name, section):
    p = params(rundir)
    assert name not in p, "Cannot extend params.json with {}, property already exists.".format(name)
    p[name] = section
    with open(os.path.join(rundir, "params.json"), "w") as f:
        json.dump(p, f, indent=4)
    return True
