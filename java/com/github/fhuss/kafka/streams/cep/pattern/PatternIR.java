/*
 * PatternIR.java -- lowers a reference Pattern (the QueryBuilder/Pattern DSL, unchanged) to the byte IR
 * libkcep.so compiles, or says why it cannot: the per-query half of the drop-in boundary (SURVEY.md
 * §8(b): "lambdas the IR cannot express fall back to the reference CPU path").
 *
 * It lives in the reference's package because the Pattern accessors it reads are package-private
 * (Pattern.java:130-213).  The walk follows the ancestor chain first to last (Pattern.iterator walks
 * last to first, Pattern.java:216-239), and issues one IR-builder call per DSL element over JNI
 * (jni/kcep_jni.c -> cep_irb_* of include/kcep.h):
 *
 *   select(name | null, level, strategy | null, topic | null)   Pattern fields :42-62, Selected.java
 *   quantifier(oneOrMore, optional, times)                      StageBuilder / PredicateBuilder
 *   within(unit.toMillis(time))                                 PatternBuilder.within
 *   <matcher tree> then where                                   Pattern.andPredicate / orPredicate :157-169
 *   <aggregate> then fold(state, type)                          PatternBuilder.fold -> StateAggregator
 *
 * A matcher tree is lowerable when every leaf carries its body (Ir.Carrying: Ir.simple / stateful /
 * sequence) and every inner node is one of the reference's own combinators -- Matcher.AndPredicate /
 * OrPredicate / NotPredicate (Matcher.java:52-103, children read reflectively: they are private), or
 * TruePredicate / TopicPredicate.  An aggregator is lowerable when it is an Ir.IrAggregator.  Anything
 * else is an opaque lambda: encode() returns a CPU decision with the reason, and the query runs on the
 * reference CEPProcessor.  A lowered IR that no device path accepts (cep_compile + cep_pattern_check)
 * is routed the same way, so that the reference raises its own InvalidPatternException.
 *
 * The Pattern's own name and level are read reflectively too (there is no getLevel(), and getName()
 * turns a null name into the level's digits, Pattern.java:181-183): the IR carries both, exactly as
 * kafkastreams-cep_amd/kcep/pattern.py encode_pattern writes them, so both hosts produce the same bytes.
 *
 * NOT BUILT in this repository (no JDK in the image, SURVEY.md §8c).  tests/patternir_twin.py restates
 * encode() call for call over the compiled JNI shim (against a stub jni.h) and checks the bytes against
 * Pattern.to_ir for every golden fixture and BASELINE config (tests/test_patternir_cpu.py).
 */
package com.github.fhuss.kafka.streams.cep.pattern;

import com.github.fhuss.kafka.streams.cep.pattern.ir.Expr;
import com.github.fhuss.kafka.streams.cep.pattern.ir.Ir;
import com.github.fhuss.kafka.streams.cep.pattern.ir.IrSchema;

import java.lang.reflect.Field;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.Collections;
import java.util.List;

public final class PatternIR {

    static { System.loadLibrary("kcep_jni"); }      // links libkcep.so

    // ---- native entry points (jni/kcep_jni.c), one per cep_irb_* call; strings as UTF-8 bytes ----
    private static native long irbNew(int[] colTypes);                                          // cep_irb_new
    private static native void irbFree(long b);                                                 // cep_irb_free
    private static native int irbTopic(long b, byte[] topic);                                   // cep_irb_topic
    private static native int irbSelect(long b, byte[] name, int level, int strategy, byte[] topic); // cep_irb_select
    private static native int irbQuantifier(long b, int oneOrMore, int optional, int times);    // cep_irb_quantifier
    private static native int irbWithin(long b, long windowMs);                                 // cep_irb_within
    private static native int irbConst(long b, int type, long i, double d);                     // cep_irb_const
    private static native int irbField(long b, int column);                                     // cep_irb_field
    private static native int irbEvent(long b, int what);                                       // cep_irb_event
    private static native int irbTopicEq(long b, byte[] topic);                                 // cep_irb_topic_eq
    private static native int irbState(long b, byte[] name, int type, int orElse);              // cep_irb_state
    private static native int irbCurr(long b, int type);                                        // cep_irb_curr
    private static native int irbSeq(long b, int kind, int column, byte[] stage);               // cep_irb_seq
    private static native int irbOp(long b, int op);                                            // cep_irb_op
    private static native int irbCast(long b, int type);                                        // cep_irb_cast
    private static native int irbWhere(long b, int conj);                                       // cep_irb_where
    private static native int irbFold(long b, byte[] state, int type);                          // cep_irb_fold
    private static native byte[] irbFinish(long b);                                             // cep_irb_finish
    private static native String[] irbTopics(long b);                                           // cep_irb_topic_name
    private static native int irbProbe(byte[] ir);                   // cep_compile + cep_pattern_check(CARRY)
    private static native String irbLastError();                                                // cep_last_error

    private static final int CEP_OK = 0, CEP_E_INVALID_PATTERN = 1, OP_AND = 0x31, OP_OR = 0x32, OP_NOT = 0x30;

    /** The per-query decision: the IR and the topic ids it uses (GPU), or why the query stays on the CPU. */
    public static final class Lowered {
        public final byte[] ir;                  // null: run the reference CEPProcessor
        public final List<String> topics;        // topic id i = topics.get(i) (the processor's interning)
        public final String reason;
        public final int status;                 // kcep status of the probe (0 when lowered)
        private Lowered(byte[] ir, List<String> topics, String reason, int status) {
            this.ir = ir; this.topics = topics; this.reason = reason; this.status = status;
        }
        public boolean gpu() { return ir != null; }
        static Lowered cpu(String why, int status) { return new Lowered(null, Collections.emptyList(), why, status); }
    }

    /** signals an opaque leaf during the walk */
    private static final class Opaque extends Exception {
        Opaque(String why) { super(why, null, false, false); }
    }

    private PatternIR() {}

    /** Lowers the chain ending at `last` (the Pattern build() returned) over the value schema. */
    public static <K, V> Lowered encode(Pattern<K, V> last, IrSchema<V> schema) {
        List<Pattern<K, V>> chain = new ArrayList<>();
        for (Pattern<K, V> p : last) chain.add(p);
        Collections.reverse(chain);
        final long b = irbNew(schema.columnTypes());
        if (b < 0) return Lowered.cpu(irbLastError(), (int) -b);
        try {
            for (String t : schema.topics()) irbTopic(b, utf8(t));
            for (Pattern<K, V> p : chain) {
                Selected sel = p.getSelected();
                Strategy st = sel.getStrategy();
                check(irbSelect(b, utf8(ownName(p)), ownLevel(p), st == null ? -1 : st.ordinal(), utf8(sel.getTopic())));
                check(irbQuantifier(b, p.getCardinality() == Pattern.Cardinality.ONE_OR_MORE ? 1 : 0,
                                    p.isOptional() ? 1 : 0, p.getTimes()));
                if (p.getWindowTime() != null)
                    check(irbWithin(b, p.getWindowUnit().toMillis(p.getWindowTime())));
                if (p.getPredicate() != null) {
                    matcher(b, p.getPredicate(), schema, p.getName());
                    check(irbWhere(b, 1));
                }
                for (StateAggregator<K, V, Object> a : p.getAggregates()) {
                    Aggregator<K, V, Object> ag = a.getAggregate();
                    if (!(ag instanceof Ir.IrAggregator))
                        throw new Opaque("fold '" + a.getName() + "' of stage " + p.getName() + " is an opaque Aggregator");
                    Ir.IrAggregator<K, V, Object> ia = (Ir.IrAggregator<K, V, Object>) ag;
                    ia.bind(schema);
                    ia.expr().emitTo(lowering(b, schema));
                    check(irbFold(b, utf8(a.getName()), ia.resultType()));
                }
            }
            byte[] ir = irbFinish(b);
            if (ir == null) return Lowered.cpu(irbLastError(), -1);
            List<String> topics = new ArrayList<>();
            Collections.addAll(topics, irbTopics(b));
            int rc = irbProbe(ir);
            if (rc != CEP_OK)                              // CEP_E_INVALID_PATTERN: the reference throws its own
                return Lowered.cpu(irbLastError(), rc);
            return new Lowered(ir, Collections.unmodifiableList(topics), null, CEP_OK);
        } catch (Opaque o) {
            return Lowered.cpu(o.getMessage(), -1);
        } catch (BuilderError e) {
            return Lowered.cpu(e.getMessage(), e.status);
        } finally {
            irbFree(b);
        }
    }

    /** Binds every Ir matcher / aggregator of the chain to the schema, whichever path the query takes:
     *  on the CPU route they evaluate their bodies against it (encode() stops at the first opaque leaf). */
    public static <K, V> void bind(Pattern<K, V> last, IrSchema<V> schema) {
        for (Pattern<K, V> p : last) {
            if (p.getPredicate() != null) bindTree(p.getPredicate(), schema);
            for (StateAggregator<K, V, Object> a : p.getAggregates())
                if (a.getAggregate() instanceof Ir.Carrying) ((Ir.Carrying) a.getAggregate()).bind(schema);
        }
    }

    private static <K, V> void bindTree(Matcher<K, V> m, IrSchema<V> schema) {
        if (m instanceof Ir.Carrying) {
            ((Ir.Carrying) m).bind(schema);
        } else if (m instanceof Matcher.AndPredicate || m instanceof Matcher.OrPredicate) {
            bindTree(child(m, "left"), schema);
            bindTree(child(m, "right"), schema);
        } else if (m instanceof Matcher.NotPredicate) {
            bindTree(child(m, "predicate"), schema);
        }
    }

    // ---- the matcher tree ----
    private static <K, V> void matcher(long b, Matcher<K, V> m, IrSchema<V> schema, String stage) throws Opaque {
        if (m instanceof Ir.Carrying) {
            ((Ir.Carrying) m).bind(schema);
            ((Ir.Carrying) m).expr().emitTo(lowering(b, schema));
        } else if (m instanceof Matcher.AndPredicate || m instanceof Matcher.OrPredicate) {
            matcher(b, child(m, "left"), schema, stage);
            matcher(b, child(m, "right"), schema, stage);
            check(irbOp(b, m instanceof Matcher.AndPredicate ? OP_AND : OP_OR));
        } else if (m instanceof Matcher.NotPredicate) {
            matcher(b, child(m, "predicate"), schema, stage);
            check(irbOp(b, OP_NOT));
        } else if (m instanceof Matcher.TruePredicate) {
            check(irbConst(b, Expr.BOOL, 1, 0));
        } else if (m instanceof Matcher.TopicPredicate) {
            check(irbTopicEq(b, utf8((String) read(m, Matcher.TopicPredicate.class, "topic"))));
        } else {
            throw new Opaque("stage " + stage + " has an opaque matcher (" + m.getClass().getName() + ")");
        }
    }

    @SuppressWarnings("unchecked")
    private static <K, V> Matcher<K, V> child(Matcher<K, V> m, String field) {
        return (Matcher<K, V>) read(m, m.getClass(), field);
    }

    private static Object read(Object o, Class<?> c, String field) {
        try {
            Field f = c.getDeclaredField(field);
            f.setAccessible(true);
            return f.get(o);
        } catch (ReflectiveOperationException e) {
            throw new IllegalStateException("reference class layout changed: " + c.getName() + "." + field, e);
        }
    }

    private static String ownName(Pattern<?, ?> p) { return (String) read(p, Pattern.class, "name"); }
    private static int ownLevel(Pattern<?, ?> p) { return (Integer) read(p, Pattern.class, "level"); }

    // ---- Expr.Lowering over the builder ----
    private static Expr.Lowering lowering(final long b, final IrSchema<?> schema) {
        return new Expr.Lowering() {
            public void constant(int type, long i, double d) { check(irbConst(b, type, i, d)); }
            public void field(int column) { check(irbField(b, column)); }
            public void event(int what) { check(irbEvent(b, what)); }
            public void topicEq(String topic) { check(irbTopicEq(b, utf8(topic))); }
            public void state(String name, int type, boolean orElse) { check(irbState(b, utf8(name), type, orElse ? 1 : 0)); }
            public void curr(int type) { check(irbCurr(b, type)); }
            public void seq(int kind, int column, String stage) { check(irbSeq(b, kind, column, utf8(stage))); }
            public void op(int op) { check(irbOp(b, op)); }
            public void cast(int type) { check(irbCast(b, type)); }
            public int column(String name) { return schema.column(name); }
        };
    }

    /** a builder call failed: the body is not typed as the IR requires (CEP_E_BAD_IR) */
    private static final class BuilderError extends RuntimeException {
        final int status;
        BuilderError(int status, String msg) { super(msg); this.status = status; }
    }

    private static void check(int rc) {
        if (rc != CEP_OK) throw new BuilderError(rc, irbLastError());
    }

    private static byte[] utf8(String s) { return s == null ? null : s.getBytes(StandardCharsets.UTF_8); }
}
