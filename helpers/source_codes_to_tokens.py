#!/usr/bin/env python
"""CLI-compatible entry point (same flags as the reference script); see ``serann.cli.tools.source_codes_to_tokens_main``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    from serann.cli.tools import source_codes_to_tokens_main
    source_codes_to_tokens_main()
