"""TimeService client (reference: Code/gRPC/client.py — one unary call to a hard-wired
192.168.1.101:50051, no deadline or retry).  Here the address is a flag, and the call has a
deadline with bounded retries.

    python -m edgellm.cli.client --address 127.0.0.1:50051
"""
from __future__ import annotations

import argparse
from typing import List, Optional

from ..serve.time_service import get_current_time


def main(argv: Optional[List[str]] = None) -> str:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--address", default="127.0.0.1:50051")
    ap.add_argument("--timeout", type=float, default=5.0, help="per-attempt deadline (s)")
    ap.add_argument("--retries", type=int, default=3)
    a = ap.parse_args(argv)
    t = get_current_time(a.address, timeout=a.timeout, retries=a.retries)
    print(f"Current Time from {a.address}: {t}")
    return t


if __name__ == "__main__":
    main()
