"""python -m allsteps_isaaclab_amd.compat <script.py> [args...]: run a reference script with the shims."""

import sys

from . import run_script

if len(sys.argv) < 2:
    raise SystemExit(__doc__)
run_script(sys.argv[1], sys.argv[2:])
