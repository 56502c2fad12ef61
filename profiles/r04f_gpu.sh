cd $ROOT
timeout -k 10 300 python3 profiles/probe.py --config c3 --rounds 3 --frames 20 --cases 'base;IRT_QUEUE=1;IRT_QUEUE=1,IRT_QUEUE_WGS=2' \
  > $O/probe_queue_c3.jsonl 2> $O/probe_queue_c3.err || exit 1
