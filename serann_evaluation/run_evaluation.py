#!/usr/bin/env python
"""CLI-compatible entry point: ``python serann_evaluation/run_evaluation.py -p ... -n ...``.
See ``serann.cli.run_evaluation``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    from serann.cli.run_evaluation import main
    main(script=os.path.abspath(__file__))
