// A/B policy variant hs16 (tools/ab_build.sh hs16 -DELECT_EC_POLICY_HEADER=...)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.hashed_scalar_waves = 16;
    return p;
}();
