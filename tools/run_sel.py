"""pytest with the arguments written in a file (shell-quoted), for GPU runs whose selection
would not survive nested quoting: python tools/run_sel.py ARGFILE [extra pytest args]."""
import shlex
import sys

import pytest

sys.exit(pytest.main(shlex.split(open(sys.argv[1]).read()) + sys.argv[2:]))
