// A/B policy variant hashfuse: assign-mode hashes finalized by each unit's last wave (hash_finalize), no hash_reduce
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.hash_fused_finalize = true;
    return p;
}();
