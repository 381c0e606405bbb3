#!/usr/bin/env python
"""CLI-compatible entry point: ``python evolutionary_experiment/run_experiment.py --parameters=...``.
See ``serann.cli.run_experiment``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    from serann.cli.run_experiment import main
    main(script=os.path.abspath(__file__))
