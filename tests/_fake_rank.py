"""Stand-in worker for tests/test_bench_launch.py: behaves like one bench.py rank as far as the
launcher sees it (environment in, a log line on stderr, rank 0's JSON line on stdout, exit
status), without touching torch or a GPU.  FAKE_RANK_FAIL=r makes rank r exit 3;
FAKE_RANK_NGPUS overrides the n_gpus rank 0 reports; FAKE_RANK_HANG=r makes rank r sleep
(a rank stuck in a collective)."""
import json
import os
import sys
import time

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
print(f"rank {rank}/{world} local {os.environ['LOCAL_RANK']} master "
      f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']} args {sys.argv[1:]}",
      file=sys.stderr, flush=True)
if os.environ.get("FAKE_RANK_FAIL") == str(rank):
    sys.exit(3)
if os.environ.get("FAKE_RANK_HANG") == str(rank):
    time.sleep(600)
if rank == 0:
    print("plain text on rank 0's stdout", flush=True)
    print(json.dumps({"metric": "fake", "n_gpus": int(os.environ.get("FAKE_RANK_NGPUS", world)),
                      "launcher": os.environ.get("JMT_LAUNCHER"),
                      "backend": os.environ.get("JMT_DIST_BACKEND")}), flush=True)
