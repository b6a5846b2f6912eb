export GPU_SESSION_STRICT=1
a=""
for r in a b; do for v in in c32 c40 c48 c32lp c40lp c48lp1; do
  if [ $v = in ]; then L=""; elif [ $v = c48lp1 ]; then L="--lib abv/libgcow_vlp1c48.so"; else L="--lib abv/libgcow_$v.so"; fi
  a="$a|150|$r$v|python tools/c5_lib_time.py $L"
done; done
IFS='|' read -ra parts <<< "${a#|}"
args=()
for ((i=0; i<${#parts[@]}; i+=3)); do args+=("${parts[i]}|${parts[i+1]}|${parts[i+2]}"); done
tools/gpu_session.sh "${args[@]}"
