"""mobile_env.core -- reference-compatible core API (plugins, entities, MComCore facade) over
the MI355X step engine."""
