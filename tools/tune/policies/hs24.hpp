// A/B policy variant hs24 (tools/ab_build.sh hs24 -DELECT_EC_POLICY_HEADER=...)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.hashed_scalar_waves = 24;
    return p;
}();
