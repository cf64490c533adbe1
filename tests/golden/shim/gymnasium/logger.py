import sys


def warn(msg, *args, **kwargs):
    print("WARN:", msg, file=sys.stderr)
