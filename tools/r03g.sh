# A/B at C4 of the variable pass's light/heavy co-scheduling share with the 1-KiB light rows
set -u
bash tools/ab.sh r03g "base mix1 mix3"
