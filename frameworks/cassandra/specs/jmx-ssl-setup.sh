#!/bin/bash
# Secure JMX for a Cassandra node (service.jmx.enabled): run by the server task before Cassandra
# starts. The JMX password and access files and the key store arrive as DC/OS secrets in
# $MESOS_SANDBOX/jmx/; this checks them, locks their permissions down (the JVM refuses a
# password file others can read), optionally imports a trust store, and writes the JVM flags
# cassandra-env.sh picks up (JVM_EXTRA_OPTS via jmx.options).
set -euo pipefail
JMX_DIR="$MESOS_SANDBOX/jmx"
OPTS="$MESOS_SANDBOX/jmx.options"
for f in password_file access_file key_store key_store_password_file; do
  if [ ! -s "$JMX_DIR/$f" ]; then
    echo "secure JMX: secret $JMX_DIR/$f is missing or empty" >&2
    exit 1
  fi
done
chmod 0400 "$JMX_DIR/password_file" "$JMX_DIR/access_file"
KEY_PASS=$(tr -d '\n' < "$JMX_DIR/key_store_password_file")
TRUST_OPTS=""
{{#JMX_ADD_TRUST_STORE}}
TRUST_PASS=$(tr -d '\n' < "$JMX_DIR/trust_store_password_file")
TRUST_OPTS="-Djavax.net.ssl.trustStore=$JMX_DIR/trust_store -Djavax.net.ssl.trustStorePassword=$TRUST_PASS"
{{/JMX_ADD_TRUST_STORE}}
cat > "$OPTS" <<OPTIONS
-Dcom.sun.management.jmxremote.port={{JMX_PORT}}
-Dcom.sun.management.jmxremote.rmi.port={{JMX_RMI_PORT}}
-Dcom.sun.management.jmxremote.authenticate=true
-Dcom.sun.management.jmxremote.password.file=$JMX_DIR/password_file
-Dcom.sun.management.jmxremote.access.file=$JMX_DIR/access_file
-Dcom.sun.management.jmxremote.ssl=true
-Dcom.sun.management.jmxremote.registry.ssl=true
-Djavax.net.ssl.keyStore=$JMX_DIR/key_store
-Djavax.net.ssl.keyStorePassword=$KEY_PASS
$TRUST_OPTS
OPTIONS
chmod 0600 "$OPTS"
echo "secure JMX configured on port {{JMX_PORT}} (rmi {{JMX_RMI_PORT}})"
