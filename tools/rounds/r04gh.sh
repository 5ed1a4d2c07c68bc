#!/bin/bash
# r04g then r04h in one call (the pool is slow to hand out boxes)
bash tools/rounds/r04g.sh && bash tools/rounds/r04h.sh
