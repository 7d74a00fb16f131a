// A/B policy variant hs18 (tools/ab_build.sh hs18 -DELECT_EC_POLICY_HEADER=...)
constexpr LaunchPolicy kPolicy = [] {
    LaunchPolicy p;
    p.hashed_scalar_waves = 18;
    return p;
}();
