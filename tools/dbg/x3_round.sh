for wt in 5 10; do for ant in 0 1; do GNNEA_X3P_ANT=$ant GNNEA_X3_WT=$wt timeout -k 10 100 python tools/dbg/x3_modes.py | sed "s/^/wt $wt ant $ant /" || exit 1; done; done
