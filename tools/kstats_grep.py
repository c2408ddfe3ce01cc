import csv,sys
r=list(csv.DictReader(open(sys.argv[1])))
for x in r:
    n=x["Name"]
    if "moments1" in n or "final_blk" in n or "mv_" in n: print("  ", n[:50], x["Calls"], round(float(x["AverageNs"])/1e3,2))
