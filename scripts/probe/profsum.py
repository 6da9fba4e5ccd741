import json,sys
d=json.load(sys.stdin)
print(sys.argv[1], "event_ms %.3f"%d["event_ms"], {k:(round(v["segments_kcyc"]), round(v["segments_redone_mean"],1), v["segments"]) for k,v in d.items() if k.startswith("level")})
