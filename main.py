"""Reference-compatible entry point: ``python main.py --params <yaml>``."""
import sys

from dba_mod_amd.main import main

if __name__ == "__main__":
    sys.exit(main())
