"""Dev: write bench_oldorder.py (the C5 leg before the framer legs, as until round 4) next to
bench.py, for the framer slowdown experiments of DESIGN.md §2.7."""
s = open("bench.py").read()
new = '''        if not args.no_read_message:
            # before C5 (DESIGN.md §2.7: the framer's first reads in a bench process sometimes run
            # 2x slower, cause open; reads_ms shows which case a run hit)
            torch.cuda.empty_cache()
            extra["rpc_framer"] = framer_leg(args, dev)
            torch.cuda.empty_cache()
            extra["rpc_framer_split"] = framer_split_leg(args, dev)
        if not args.no_skewed:
            torch.cuda.empty_cache()
            extra["c5_skewed"] = skewed_leg(args, dev)'''
old = '''        if not args.no_skewed:
            torch.cuda.empty_cache()
            extra["c5_skewed"] = skewed_leg(args, dev)
        if not args.no_read_message:
            torch.cuda.empty_cache()
            extra["rpc_framer"] = framer_leg(args, dev)
            torch.cuda.empty_cache()
            extra["rpc_framer_split"] = framer_split_leg(args, dev)'''
assert new in s
open("bench_oldorder.py", "w").write(s.replace(new, old, 1))
