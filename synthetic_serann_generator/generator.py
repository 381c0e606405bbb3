#!/usr/bin/env python
"""CLI-compatible entry point (same flags as the reference script); see ``serann.cli.tools.generator_main``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    from serann.cli.tools import generator_main
    generator_main()
